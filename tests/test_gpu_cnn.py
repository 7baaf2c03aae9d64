"""GPU numerics of the client-batched TinyCNN kernels vs plain PyTorch fp32 (grouped conv / autograd)."""
import pytest
import torch
import torch.nn.functional as F

from qfedx_amd.models import tinycnn as tc

pytestmark = pytest.mark.gpu


def test_mfma_16x16x4_layout(cuda):
    from qfedx_amd.ops._ext import ext
    g = torch.Generator().manual_seed(0)
    A = torch.randn(16, 12, generator=g)
    B = torch.randn(12, 16, generator=g)
    D = torch.empty(256, device=cuda)
    ext().cnn_mfma_probe(A.to(cuda).contiguous(), B.to(cuda).contiguous(), D, 12)
    assert torch.allclose(D.view(16, 16).cpu(), A @ B, atol=1e-4)


def _batch(K, B, C=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    params = torch.stack([tc.init_flat(C, seed + k) for k in range(K)])
    params += 0.02 * torch.randn(params.shape, generator=g)
    X = torch.rand(K, B, 1, 28, 28, generator=g)
    X[X < 0.6] = 0.0                       # MNIST-like sparsity
    y = torch.randint(0, C, (K, B), generator=g)
    w = torch.full((K, B), 1.0 / B)
    mask = (torch.rand(K, B, 64, generator=g) >= 0.5).float() * 2.0
    return params, X, y, w, mask


@pytest.mark.parametrize("K,B", [(1, 1), (3, 5), (4, 32)])
def test_conv_forward_matches_torch(cuda, K, B):
    from qfedx_amd.ops.cnn_hip import HipTinyCNN
    params, X, y, w, mask = _batch(K, B)
    hip = HipTinyCNN(3, cuda)
    _, pool1, am1, pool2, am2 = hip.conv_forward(params.to(cuda), X.to(cuda))
    v = tc.views(params)
    h = X.reshape(K, B, 28, 28).transpose(0, 1)
    c1 = F.conv2d(h, v["conv1.weight"].reshape(K * 16, 1, 5, 5), v["conv1.bias"].reshape(-1), padding=2, groups=K)
    p1 = F.max_pool2d(F.relu(c1), 2)
    c2 = F.conv2d(p1, v["conv2.weight"].reshape(K * 32, 16, 5, 5), v["conv2.bias"].reshape(-1), padding=2, groups=K)
    p2 = F.max_pool2d(F.relu(c2), 2)
    ref1 = p1.reshape(B, K, 16 * 196).transpose(0, 1).reshape(K * B, -1)
    ref2 = p2.reshape(B, K, 32 * 49).transpose(0, 1).reshape(K * B, -1)
    assert torch.allclose(pool1.cpu(), ref1, atol=1e-4, rtol=1e-4)
    assert torch.allclose(pool2.cpu(), ref2, atol=1e-4, rtol=1e-4)
    lg = hip.logits(params.to(cuda), X.to(cuda)).cpu()
    assert torch.allclose(lg, tc.batched_forward(params, X, 3), atol=1e-4, rtol=1e-4)


@pytest.mark.parametrize("K,B,C", [(2, 3, 3), (3, 32, 3), (2, 7, 10), (2, 70, 10), (128, 40, 10)])
def test_loss_and_grads_match_autograd(cuda, K, B, C):
    # (128, 40): the backward takes 16 samples per workgroup (one per CU) and the last group holds 8
    from qfedx_amd.ops.cnn_hip import HipTinyCNN
    params, X, y, w, mask = _batch(K, B, C, seed=K + B)
    hip = HipTinyCNN(C, cuda)
    r = hip.loss_and_grads(params.to(cuda), X.to(cuda), y.to(cuda), w.to(cuda), mask.to(cuda))
    # float64 autograd: the kernels (conv2 forward on the 3-term fp16 split, fp32 elsewhere) are closer to it than
    # float32 torch is - a reference that rounds differently can flip a 2x2 max-pool argmax of a near-tie window
    # and move a whole gradient term (ops/cnn_hip.precision_check reports both errors)
    p = params.double().clone().requires_grad_(True)
    logits = tc.batched_forward(p, X.double(), C, mask.double())
    nll = F.cross_entropy(logits.reshape(-1, C), y.reshape(-1), reduction="none").reshape(K, B)
    loss = (nll * w.double()).sum(-1)
    loss.sum().backward()
    assert torch.allclose(r["loss"].cpu().double(), loss.detach(), atol=1e-4, rtol=1e-4)
    g = r["grad"].cpu().double()
    bounds = tc.layer_boundaries(C)
    for name, a, b in zip(tc.param_shapes(C), bounds[:-1], bounds[1:]):
        ref = p.grad[:, a:b]
        err = (g[:, a:b] - ref).abs().amax(-1)          # per client
        scale = ref.abs().max().item() + 1e-6
        # at most one client in 64 may hold a near-tie max-pool window whose argmax the float64 reference resolves
        # the other way (a whole routed gradient term; the 128 x 40 batch has 1 such window in 8M), never more
        # than 10x the bound
        bad = int((err > 2e-3 * scale + 1e-6).sum())
        assert bad <= K // 64 and err.max().item() <= 2e-2 * scale + 1e-6, (name, bad, err.max().item(), scale)
    acc = ((logits.argmax(-1) == y) & (w > 0)).sum(-1).float()
    assert torch.equal(r["correct"].cpu(), acc)


def test_cfed_federated_run_hip_matches_cpu(cuda):
    from qfedx_amd.api import run_experiment
    from qfedx_amd.config import ExperimentConfig
    from qfedx_amd.parallel.dist import init_distributed

    def cfg(dev, backend):
        c = ExperimentConfig()
        c.model.kind = "tinycnn"
        c.data.num_clients = 4
        c.data.samples_per_client = 64
        c.data.test_samples = 128
        c.train.num_rounds = 2
        c.train.optimizer = "sgd"
        c.train.learning_rate = 0.05
        c.train.batch_size = 16
        c.train.aggregate = "weights"
        c.train.wrap_angles = False
        c.runtime.device = dev
        c.runtime.backend = backend
        c.runtime.log_every = 100
        return c

    cpu = run_experiment(cfg("cpu", "torch"))
    dev = torch.device("cuda", 0)
    gpu = run_experiment(cfg("cuda", "hip"), world=init_distributed(dev), device=dev, backend="hip")
    assert torch.allclose(gpu["params"].cpu(), cpu["params"], atol=2e-4, rtol=1e-3)
    assert abs(gpu["accuracies"][-1] - cpu["accuracies"][-1]) < 0.02


@pytest.mark.parametrize("local_epochs,momentum", [(1, 0.9), (2, 0.5)])
def test_cfed_fused_sgd_step_bitwise(cuda, local_epochs, momentum):
    """The SGD-momentum step fused into the gradient-producing kernels (cnn_args.h; the first local step reading theta
    broadcast, no row init, no gradient buffer, no optimizer launch) is bitwise the separate qfx_sgdm launch: several
    local steps with unequal non-IID shards (rows going inactive), momentum carried across steps."""
    from qfedx_amd.api import run_experiment
    from qfedx_amd.config import ExperimentConfig
    from qfedx_amd.parallel.dist import init_distributed

    def cfg(fuse):
        c = ExperimentConfig()
        c.model.kind = "tinycnn"
        c.data.num_clients = 5
        c.data.samples_per_client = 48
        c.data.partition_type = "non_iid"
        c.data.test_samples = 64
        c.train.num_rounds = 2
        c.train.local_epochs = local_epochs
        c.train.optimizer = "sgd"
        c.train.momentum = momentum
        c.train.learning_rate = 0.05
        c.train.batch_size = 16
        c.train.aggregate = "weights"
        c.train.wrap_angles = False
        c.train.fuse_optimizer = fuse
        c.runtime.device = "cuda"
        c.runtime.backend = "hip"
        c.runtime.log_every = 100
        return c

    dev = torch.device("cuda", 0)
    a = run_experiment(cfg(True), world=init_distributed(dev), device=dev, backend="hip")
    b = run_experiment(cfg(False), world=init_distributed(dev), device=dev, backend="hip")
    assert torch.equal(a["params"], b["params"])
    assert a["accuracies"] == b["accuracies"]
    assert [h["train_loss"] for h in a["history"]] == [h["train_loss"] for h in b["history"]]
    assert max(h["local_steps"] for h in a["history"]) > 5         # several steps per client per round


def test_head_dropout_from_uniforms_matches_mask(cuda):
    """The head drawing the inverted-dropout mask from the clients' Philox keys gives bit-identical results to the
    materialised ``dropout_masks`` tensor."""
    from qfedx_amd.ops.cnn_hip import HipTinyCNN
    K, B, C = 3, 20, 10
    params, X, y, w, _ = _batch(K, B, C, seed=5)
    hip = HipTinyCNN(C, cuda)
    ids = [7, 11, 19]
    keys = tc.dropout_keys(ids, 42, 3).to(cuda)
    m = tc.dropout_masks(ids, B, 42, 3, 1, cuda)
    args = (params.to(cuda), X.to(cuda), y.to(cuda), w.to(cuda))
    r1 = hip.loss_and_grads(*args, m)
    r1 = {k: v.clone() for k, v in r1.items()}
    r2 = hip.loss_and_grads(*args, ("philox", keys, 1, 0.5))
    for k in ("loss", "grad", "correct"):
        assert torch.equal(r1[k], r2[k]), k
