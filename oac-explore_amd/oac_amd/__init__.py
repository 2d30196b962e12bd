"""oac_amd -- MI355X-native OAC/SAC gradient-step hot path.

Drop-in replacements for the reference's hot-path interfaces:
  SACTrainer                         trainer/trainer.py
  ParticleTrainer                    trainer/particle_trainer.py (p-oac recipes, share_layers)
  ParticleTrainerOAC                 trainer/particle_trainer_oac.py (share_layers)
  GaussianTrainer                    trainer/gaussian_trainer.py (g-oac, share_layers)
  get_optimistic_exploration_action  optimistic_exploration.py
  ReplayBuffer, ReplayBufferCount    replay_buffer.py
  vec_rollout                        path_collector.py rollout over N envs, one call per step
backed by liboac_amd.so (hand-written HIP for gfx950 behind a C ABI).
"""
from ._lib import lib, LIB_PATH  # noqa: F401
from .trainer import SACTrainer, row_layout  # noqa: F401
from .particle_trainer import ParticleTrainer  # noqa: F401
from .particle_trainer_oac import ParticleTrainer as ParticleTrainerOAC  # noqa: F401
from .gaussian_trainer import GaussianTrainer  # noqa: F401
from .replay_buffer import ReplayBuffer, ReplayBufferCount, DeviceBatch, DeviceIndexStream  # noqa: F401
from .optimistic_exploration import (get_optimistic_exploration_action,  # noqa: F401
                                     get_optimistic_exploration_actions)
from .producers import get_policy_producer, get_q_producer  # noqa: F401
from .networks import MakeDeterministic  # noqa: F401
from .rollout import vec_rollout  # noqa: F401
