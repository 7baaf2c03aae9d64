"""Data layer: IDX I/O, preprocessing split sizes, partitioner parity with the reference, features."""
import importlib.util
import os
import random
import sys

import numpy as np
import pytest
import torch

from qfedx_amd.data import (create_iid_partition, create_non_iid_partition, downsample_batch, downsample_image,
                            pool_batch, pool_to_n_features, preprocess_mnist, read_idx_images, read_idx_labels,
                            write_idx_images, write_idx_labels, write_synthetic_mnist, StandardPCA, partition,
                            class_distribution, load_iris_federated, load_synthetic_federated)

REF = "/root/reference"


def _load_ref(mod_path, name):
    """Import a reference module read-only (behaviour parity tests; nothing is copied)."""
    if not os.path.exists(mod_path):
        pytest.skip("reference not mounted")
    sys.dont_write_bytecode = True
    d = os.path.dirname(mod_path)
    if d not in sys.path:
        sys.path.insert(0, d)
    spec = importlib.util.spec_from_file_location(name, mod_path)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_idx_roundtrip(tmp_path):
    imgs = np.random.default_rng(0).integers(0, 255, (7, 28, 28)).astype(np.uint8)
    labs = np.arange(7, dtype=np.uint8)
    write_idx_images(str(tmp_path / "i.idx"), imgs)
    write_idx_labels(str(tmp_path / "l.idx"), labs)
    assert np.array_equal(read_idx_images(str(tmp_path / "i.idx")), imgs)
    assert np.array_equal(read_idx_images(str(tmp_path / "i.idx"), strict=True), imgs)
    assert np.array_equal(read_idx_labels(str(tmp_path / "l.idx"), strict=True), labs)


def test_reference_label_files_parse():
    p = os.path.join(REF, "dataset/raw/train-labels.idx1-ubyte")
    if not os.path.exists(p):
        pytest.skip("reference labels absent")
    y = read_idx_labels(p, strict=True)
    assert y.shape == (60000,) and y.max() == 9


@pytest.fixture(scope="module")
def synth_raw(tmp_path_factory):
    d = tmp_path_factory.mktemp("mnist")
    src = os.path.join(REF, "dataset/raw") if os.path.isdir(os.path.join(REF, "dataset/raw")) else None
    write_synthetic_mnist(str(d / "raw"), src, seed=0)
    return d, src is not None


def test_preprocess_split_sizes_match_reference(synth_raw):
    d, real_labels = synth_raw
    random.seed(42)
    np.random.seed(42)
    out = preprocess_mnist(str(d / "raw"), str(d / "proc"), results_folder=str(d / "res"), plots=False,
                           verbose=False)
    train, val, test, clients = out
    assert train[0].dtype == torch.float32 and train[0].shape[1:] == (1, 28, 28)
    assert train[1].dtype == torch.int64
    if real_labels:   # 16 760 / 1 863 / 3 147, 4 190 per IID client
        assert (len(train[1]), len(val[1]), len(test[1])) == (16760, 1863, 3147)
        assert [len(c[1]) for c in clients] == [4190] * 4
    # fixed quirk #1: client shards are tensors with int64 labels (reference crashed on numpy)
    assert isinstance(clients[0][0], torch.Tensor) and clients[0][1].dtype == torch.int64
    # bit-compatible saved layout, loadable with weights_only
    X, y = torch.load(str(d / "proc" / "train.pt"), weights_only=True)
    assert X.shape == train[0].shape and y.dtype == torch.int64


def test_preprocess_missing_files_returns_none(tmp_path, capsys):
    assert preprocess_mnist(str(tmp_path / "nope"), str(tmp_path / "p"), plots=False) is None


def test_iid_partition_parity_with_reference():
    ref = _load_ref(os.path.join(REF, "src/CFed/Preprocess.py"), "ref_preprocess")
    X = np.arange(103 * 2).reshape(103, 2)
    y = (np.arange(103) % 3).astype(np.uint8)
    random.seed(7)
    a = ref.create_iid_partition(X, y, 4)
    random.seed(7)
    b = create_iid_partition(X, y, 4)
    for (xa, ya), (xb, yb) in zip(a, b):
        assert np.array_equal(xa, xb) and np.array_equal(ya, yb)
    assert [len(p[1]) for p in b] == [25, 25, 25, 28]   # remainder to the last client


def test_non_iid_partition_parity_and_label_fix():
    ref = _load_ref(os.path.join(REF, "src/CFed/Preprocess.py"), "ref_preprocess")
    X = np.arange(300).reshape(300, 1)
    y = (np.arange(300) % 3).astype(np.uint8)
    random.seed(3)
    np.random.seed(3)
    a = ref.create_non_iid_partition(X, y, 5, 0.5)
    random.seed(3)
    np.random.seed(3)
    b = create_non_iid_partition(X, y, 5, 0.5)
    for (xa, ya), (xb, yb) in zip(a, b):   # identical for contiguous labels {0..C-1}
        assert np.array_equal(xa, xb) and np.array_equal(ya, yb)
    # digits (3, 5) - the reference keeps nothing, the fixed version keeps all
    y35 = np.where(np.arange(200) % 2 == 0, 3, 5).astype(np.uint8)
    X35 = np.arange(200).reshape(200, 1)
    random.seed(1)
    np.random.seed(1)
    assert sum(len(p[1]) for p in ref.create_non_iid_partition(X35, y35, 4)) == 0
    random.seed(1)
    np.random.seed(1)
    assert sum(len(p[1]) for p in create_non_iid_partition(X35, y35, 4)) == 200


def test_unknown_partition_type_raises():
    with pytest.raises(ValueError):
        partition(np.zeros((4, 1)), np.zeros(4), 2, "weird")


def test_pool_and_downsample_rules():
    # reference downsample/pool live in qAngle.py / testEncoder.py, which import qiskit at module
    # import (unavailable here); the functions are pure numpy, so their documented rules
    # (testEncoder.py:20-56, qAngle.py:9-24) are pinned directly - parity unpinned by execution
    rng = np.random.default_rng(0)
    img = rng.random((28, 28))
    ds = downsample_image(img, (4, 4))
    assert np.allclose(ds[0, 0], img[0:7, 0:7].mean())
    assert np.allclose(downsample_batch(torch.from_numpy(img)[None], (4, 4))[0].numpy(), ds.reshape(-1))
    v = rng.random(16)
    p = pool_to_n_features(v, 5)               # chunk 3, last chunk absorbs the remainder
    assert np.allclose(p[:4], [v[0:3].mean(), v[3:6].mean(), v[6:9].mean(), v[9:12].mean()])
    assert np.isclose(p[4], v[12:].mean())
    assert np.allclose(pool_to_n_features(v[:3], 5), [v[0], v[1], v[2], 0, 0])   # zero pad
    assert np.allclose(pool_batch(torch.from_numpy(v)[None], 5)[0].numpy(), p)


def test_standard_pca_roundtrip(tmp_path):
    X = torch.randn(200, 30, dtype=torch.float64)
    t = StandardPCA(4).fit(X)
    f = t.transform(X)
    assert f.shape == (200, 4) and float(f.min()) >= 0 and float(f.max()) <= 1
    t.save(str(tmp_path / "pca.pt"))
    t2 = StandardPCA.load(str(tmp_path / "pca.pt"))
    assert torch.allclose(t2.transform(X), f)


def test_class_distribution_matrix():
    cd = [(np.zeros(3), np.array([0, 1, 1])), (np.zeros(2), np.array([2, 2]))]
    classes, dist = class_distribution(cd)
    assert classes == [0, 1, 2] and dist.tolist() == [[1, 0], [2, 0], [0, 2]]


def test_iris_and_synthetic_loaders():
    d = load_iris_federated(3, "non_iid", 0.5, seed=0)
    assert d.n_features == 4 and len(d.clients) == 3 and sum(d.sizes()) == 105
    s1 = load_synthetic_federated(8, 4, 3, 50, 64, clients=[2, 5])
    s2 = load_synthetic_federated(8, 4, 3, 50, 64, clients=[5])
    assert torch.equal(s1.clients[1][0], s2.clients[0][0])   # shard independent of which rank builds it
