"""Reference-API compatibility layer (qfedx_amd.compat): names, signatures, return shapes."""
import numpy as np
import torch

from qfedx_amd.compat import Classical_FL, Preprocess, qAmplitude, qAngle, testEncoder
from qfedx_amd.data.synthetic import synthetic_digit_images


def _shards(n_clients=2, n=40, C=3, seed=0):
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n_clients):
        y = rng.integers(0, C, size=n).astype(np.int64)
        X = synthetic_digit_images(y, seed + k).astype(np.float32)[:, None] / 255.0
        out.append((X, y))          # numpy shards, as Preprocess returns them (reference C16 crash)
    return out


def test_reference_names_exist():
    for mod, names in [(Preprocess, ["read_idx_images", "read_idx_labels", "create_iid_partition",
                                      "create_non_iid_partition", "visualize_client_data",
                                      "plot_class_distribution", "preprocess_mnist", "main"]),
                       (Classical_FL, ["set_seeds", "TinyCNN", "client_update", "federated_averaging",
                                       "evaluate_model", "federated_learning", "main"]),
                       (qAmplitude, ["normalize_for_amplitude", "amplitude_encode", "get_statevector_from_circuit"]),
                       (qAngle, ["pool_to_n_features", "angle_encode"]),
                       (testEncoder, ["downsample_image", "pool_to_n_features", "main"])]:
        for n in names:
            assert callable(getattr(mod, n)), (mod.__name__, n)


def test_client_update_returns_state_dict_and_count():
    torch.manual_seed(0)
    m = Classical_FL.TinyCNN(3)
    sd0 = {k: v.clone() for k, v in m.state_dict().items()}
    X, y = _shards(1, 40)[0]
    sd, n = Classical_FL.client_update(sd0, (X, y), epochs=1, lr=0.05, batch_size=16)
    assert n == 40 and list(sd.keys()) == list(sd0.keys())
    assert all(sd[k].shape == sd0[k].shape for k in sd)
    assert any(not torch.equal(sd[k], sd0[k]) for k in sd)


def test_federated_learning_shapes_and_learning():
    shards = _shards(2, 60)
    yt = np.arange(90) % 3
    test = (synthetic_digit_images(yt, 99).astype(np.float32)[:, None] / 255.0, yt)
    out = Classical_FL.federated_learning(shards, test, num_rounds=3, local_epochs=1, learning_rate=0.05,
                                          batch_size=16, num_classes=3, log_every=100)
    assert set(out) >= {"model", "accuracies"}
    assert len(out["accuracies"]) == 4                         # round 0 + 3 rounds (Classical_FL.py:116-148)
    assert isinstance(out["model"], torch.nn.Module)
    acc = Classical_FL.evaluate_model(out["model"].cpu(), test)
    assert abs(acc - out["accuracies"][-1]) < 1e-6
    assert out["accuracies"][-1] > out["accuracies"][0]


def test_encoder_demo_runs_on_synthetic_image(tmp_path):
    img = synthetic_digit_images(np.array([2]), 3)[0]
    res = testEncoder.main(image=img, verbose=False, results_folder=str(tmp_path))
    assert res["downsampled"].shape == (4, 4)
    assert len(res["amplitudes"]) == 8
    assert res["amplitude_circuit"].name == "AmplitudeEncode"
    assert res["angle_circuit"].name == "AngleEncode_RY"
