"""Utilities package (mirror of reference src/utils/__init__.py, hot-path subset)."""
from .activation import get_activation_function
from .distributed import is_main_process, safe_get_rank

__all__ = ["is_main_process", "safe_get_rank", "get_activation_function"]
