"""imitation_amd: MI355X-native imitation and reward learning.

Public API mirrors the reference ``imitation`` package (``algorithms``, ``data``,
``policies``, ``rewards``, ``regularization``, ``util``, ``scripts``); the RL
substrate it needs (PPO/SAC/DQN, policies, VecEnvs, logger) lives in
:mod:`imitation_amd.rl` and :mod:`imitation_amd.envs`; HIP/CDNA4 kernels are in
``csrc/`` and exposed through :mod:`imitation_amd.ops`.
"""

__version__ = "0.1.0"
