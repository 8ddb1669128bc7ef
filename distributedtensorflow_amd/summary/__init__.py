"""Observability: reference-compatible logger API and native TensorBoard event files."""
from . import logger
from .events import EventFileWriter, FileWriter, event_files, read_scalars, summary_iterator

__all__ = ["logger", "EventFileWriter", "FileWriter", "event_files", "read_scalars",
           "summary_iterator"]
