"""Training orchestration: global step, hooks, MonitoredTrainingSession, Supervisor, Saver."""
from .global_step import (GlobalStep, create_global_step, get_global_step,
                          get_or_create_global_step, reset_global_step)

__all__ = ["GlobalStep", "create_global_step", "get_global_step", "get_or_create_global_step",
           "reset_global_step"]
