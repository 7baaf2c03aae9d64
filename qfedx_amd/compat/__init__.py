"""Reference-API compatibility layer: the public functions of the reference's modules under their
original module and function names, running on this framework's engine.

    from qfedx_amd.compat import Classical_FL, Preprocess, qAmplitude, qAngle, testEncoder

* ``Preprocess``   - ``src/CFed/Preprocess.py``   (IDX readers, partitioners, plots, preprocess_mnist)
* ``Classical_FL`` - ``src/CFed/Classical_FL.py`` (set_seeds, TinyCNN, client_update,
  federated_averaging, evaluate_model, federated_learning, main)
* ``qAmplitude``   - ``src/QFed/qAmplitude.py``   (normalize_for_amplitude, amplitude_encode,
  get_statevector_from_circuit)
* ``qAngle``       - ``src/QFed/qAngle.py``       (pool_to_n_features, angle_encode)
* ``testEncoder``  - ``src/QFed/testEncoder.py``  (downsample_image, the encoder demo as ``main``)

Signatures and return shapes follow the reference; the documented reference bugs are fixed
(numpy client shards are accepted, ``num_classes`` is not hard-coded, Dirichlet partition keys by
the actual labels, ``main()`` runs end to end) - see SURVEY.md §2.1 / §8.
"""
from . import Classical_FL, Preprocess, qAmplitude, qAngle, testEncoder  # noqa: F401
