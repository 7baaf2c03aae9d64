"""CFed conv kernels vs float64 torch on the test_gpu_cnn (K=2, B=70, C=10) batch: pool2 error and how many 2x2
max-pool argmaxes / ReLU states differ from float64 (kernel and float32 torch).  QFX_PKG_ROOT selects the tree."""
import os
import sys
sys.path.insert(0, os.environ.get("QFX_PKG_ROOT") or os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(1, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import json
import torch
import torch.nn.functional as F
from qfedx_amd.models import tinycnn as tc
from qfedx_amd.ops.cnn_hip import HipTinyCNN, precision_check
from tests.test_gpu_cnn import _batch

dev = torch.device("cuda", 0)
out = {}
for (K, B, C) in ((2, 70, 10), (128, 40, 10)):
    params, X, y, w, mask = _batch(K, B, C, seed=K + B)
    hip = HipTinyCNN(C, dev)
    _, p1, a1, p2, a2 = hip.conv_forward(params.to(dev), X.to(dev))
    v = tc.views(params.double(), C)
    h = X.double().reshape(K, B, 28, 28).transpose(0, 1)
    c1 = F.conv2d(h, v["conv1.weight"].reshape(K * 16, 1, 5, 5), v["conv1.bias"].reshape(-1), padding=2, groups=K)
    r1 = F.max_pool2d(F.relu(c1), 2)
    c2 = F.conv2d(r1, v["conv2.weight"].reshape(K * 32, 16, 5, 5), v["conv2.bias"].reshape(-1), padding=2, groups=K)
    r2, i2 = F.max_pool2d(F.relu(c2), 2, return_indices=True)
    ref2 = r2.reshape(B, K, 32 * 49).transpose(0, 1).reshape(K * B, -1)
    k2 = p2.double().cpu()
    # argmax code 0..3 of the float64 reference per window
    ix = i2.reshape(B, K, 32, 49)
    wy = torch.arange(49) // 7
    wx = torch.arange(49) % 7
    yy, xx = ix // 14, ix % 14
    code = ((yy - 2 * wy) * 2 + (xx - 2 * wx)).transpose(0, 1).reshape(K * B, -1)
    am = a2.long().cpu()
    pos = ref2 > 0
    out[f"{K}x{B}"] = {"max_abs_err_pool2": float((k2 - ref2).abs().max()), "max_pool2": float(ref2.abs().max()),
                       "argmax_mismatch_active_windows": int(((am != code) & pos).sum()),
                       "relu_state_mismatch": int(((k2 > 0) != pos).sum()), "windows": int(ref2.numel())}
out["precision"] = precision_check(10, dev, K=2, B=70, seed=3)
print(json.dumps(out))
