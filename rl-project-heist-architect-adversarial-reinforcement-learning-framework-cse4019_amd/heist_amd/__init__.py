"""heist_amd -- MI355X-native hot path of the Heist Architect adversarial RL game.

Batched environment step/reset, layout BFS, GAE and the clipped-PPO loss run as
hand-written HIP kernels for gfx950 behind the C ABI in include/heist.h
(libheist_hip.so); this package mirrors the reference's Python API on top.
"""
__version__ = "0.1.0"

from .environment import EnvironmentConfig, HeistEnvironment  # noqa: F401
from .vec_env import HeistEnv, LayoutBatch, STATUS_NAMES  # noqa: F401
