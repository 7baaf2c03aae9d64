"""``src/QFed/qAngle.py`` API (reference ``qAngle.py:9-51``)."""
from ..data.features import pool_to_n_features  # noqa: F401
from ..quantum.encoders import angle_encode  # noqa: F401
