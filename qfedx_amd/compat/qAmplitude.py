"""``src/QFed/qAmplitude.py`` API (reference ``qAmplitude.py:11-46``): float64 CPU circuits; the
batched GPU path is ``qfedx_amd.quantum.encoders.amplitude_states`` + the statevector engine."""
from ..quantum.encoders import amplitude_encode, get_statevector_from_circuit, normalize_for_amplitude  # noqa: F401
