"""Training orchestration (TF1 ``tf.train`` surface): global step, hooks,
MonitoredTrainingSession, Supervisor, Saver / checkpoints, ConfigProto."""
from .checkpoint import (CheckpointState, Saver, checkpoint_exists, get_checkpoint_state,
                         latest_checkpoint, list_variables, load_saved_model_variables,
                         load_variable, save_saved_model, update_checkpoint_state)
from .graphed import GraphedTrainStep
from .global_step import (GlobalStep, create_global_step, get_global_step,
                          get_or_create_global_step, reset_global_step)
from .hooks import (CheckpointSaverHook, FaultInjectionHook, FinalOpsHook, InjectedFault,
                    LoggingTensorHook, NanTensorHook, SessionRunArgs, SessionRunContext,
                    SessionRunHook, SessionRunValues, StepCounterHook, StopAtStepHook,
                    SummarySaverHook)
from .session import (ConfigProto, MonitoredTrainingSession, RunConfig, Scaffold, Supervisor,
                      wait_for_new_checkpoint)

__all__ = [n for n in dir() if not n.startswith("_")]
