"""Data layer: IDX I/O, partitioners, MNIST preprocessing, features, synthetic shards, plots."""
from .idx import read_idx_images, read_idx_labels, write_idx_images, write_idx_labels
from .partition import create_iid_partition, create_non_iid_partition, dirichlet_indices, partition
from .features import (downsample_image, downsample_batch, pool_to_n_features, pool_batch,
                       angle_scale, StandardPCA, make_features)
from .mnist import preprocess_mnist, load_processed
from .viz import visualize_client_data, plot_class_distribution, class_distribution
from .synthetic import (synthetic_digit_images, write_synthetic_mnist, synthetic_client_shards,
                        synthetic_test_set, synthetic_images_shards)
from .datasets import (FederatedData, build_federated_data, load_iris_federated,
                       load_mnist_federated, load_synthetic_federated)
