"""``ray.tune.progress_reporter`` import path."""
from .registry import CLIReporter, JupyterNotebookReporter, ProgressReporter

__all__ = ["ProgressReporter", "CLIReporter", "JupyterNotebookReporter"]
