"""mhppo — MI355X-native hot path of MH-PPO (BrunoudA/MH-PPO).

Vectorised crosswalk envs, GPU rollout collector, returns scan and PPO update
as hand-written HIP kernels for gfx950 behind a C-ABI (include/mhppo.h), with
the reference's Gym env / Model_PPO / Env_rollout / Algo_PPO surface on top.
"""
from .env import VecCrosswalk  # noqa: F401

__version__ = "0.1.0"
