"""``src/QFed/testEncoder.py`` API (reference ``testEncoder.py:20-129``): ``downsample_image``,
``pool_to_n_features`` and the encoder demo as ``main`` (non-blocking: figures are saved, not shown)."""
from __future__ import annotations

import os

import numpy as np

from ..data.features import downsample_image, pool_to_n_features  # noqa: F401
from ..quantum.encoders import amplitude_encode, angle_encode, get_statevector_from_circuit
from ..utils.seeding import set_seeds


def main(raw_folder: str = "./dataset/raw", processed_folder: str = "./dataset/processed",
         results_folder: str = "./results", image: np.ndarray | None = None, verbose: bool = True) -> dict:
    """First training image -> 4x4 -> amplitude-encode 16 -> 4 qubits -> pooled RY angle encoding.

    ``image`` overrides the MNIST load (e.g. a synthetic 28x28 digit when the IDX files are absent).
    Returns the circuits, the first 8 amplitudes and the drawings (reference prints them, ``:114-127``).
    """
    set_seeds(42)
    if image is None:
        from ..data.mnist import preprocess_mnist
        out = preprocess_mnist(raw_folder, processed_folder, plots=False, verbose=verbose)
        if out is None:
            raise FileNotFoundError(f"MNIST IDX files not found under {raw_folder}")
        image = out[0][0][0, 0].numpy()
    img = np.asarray(image, dtype=np.float64).reshape(28, 28)
    small = downsample_image(img, (4, 4))
    vec = small.flatten()
    amp_qc = amplitude_encode(vec)
    sv = get_statevector_from_circuit(amp_qc)
    feats = pool_to_n_features(vec, 4)
    ang_qc = angle_encode(feats, n_qubits=4, basis="ry")
    res = {"downsampled": small, "amplitude_circuit": amp_qc, "amplitudes": sv.data[:8],
           "angle_circuit": ang_qc, "amplitude_drawing": str(amp_qc.draw("text")),
           "angle_drawing": str(ang_qc.draw("text"))}
    if verbose:
        print(res["amplitude_drawing"])
        print("First 8 amplitudes:", np.round(res["amplitudes"], 4))
        print(res["angle_drawing"])
    try:
        from ..data.viz import _plt
        plt = _plt()
        os.makedirs(results_folder, exist_ok=True)
        fig, ax = plt.subplots(1, 2, figsize=(6, 3))
        ax[0].imshow(img, cmap="gray"); ax[0].set_title("28x28")
        ax[1].imshow(small, cmap="gray"); ax[1].set_title("4x4")
        fig.savefig(os.path.join(results_folder, "encoder_demo.png"))
        plt.close(fig)
    except Exception:  # plotting is optional
        pass
    return res
