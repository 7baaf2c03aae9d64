"""``src/CFed/Preprocess.py`` API (reference ``Preprocess.py:11-247``)."""
from __future__ import annotations

from ..data.idx import read_idx_images, read_idx_labels  # noqa: F401  (C1, C2: Preprocess.py:11-20)
from ..data.mnist import preprocess_mnist  # noqa: F401  (C7: Preprocess.py:137-228)
from ..data.partition import create_iid_partition, create_non_iid_partition  # noqa: F401  (C3, C4)
from ..data.viz import plot_class_distribution, visualize_client_data  # noqa: F401  (C5, C6)
from ..utils.seeding import set_seeds


def main(raw_folder: str = "./dataset/raw", processed_folder: str = "./dataset/processed", **kw):
    """Script entry (C8, ``Preprocess.py:231-247``): seed 42, then preprocess with the defaults."""
    set_seeds(42)
    return preprocess_mnist(raw_folder, processed_folder, **kw)
