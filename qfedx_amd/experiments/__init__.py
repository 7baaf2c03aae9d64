"""Experiment grids and reporting (ROADMAP.md:102-121): sweep configs x seeds, summarise each run
(accuracy, AUC, epsilon, wall-clock, GPU-hours, communication), aggregate mean +/- std over seeds,
and draw the acc-vs-epsilon / acc-vs-qubits / speedup-vs-clients plots."""
from .grid import expand_grid, run_grid, summarize_run  # noqa: F401
from .report import aggregate, write_report  # noqa: F401
