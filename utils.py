"""Reference-compatible ``utils`` module (reference utils.py): re-exports the framework helpers.

Importing it is headless-safe (the reference ran ``stty size`` at import time)."""
from pytorch_cifar_amd.utils import (  # noqa: F401
    TOTAL_BAR_LENGTH,
    format_time,
    get_mean_and_std,
    init_params,
    progress_bar,
    set_logger,
)
