"""In-house RL substrate (the SB3 surface the reference depends on):
PPO / SAC / DQN, actor-critic policies, distributions, device-resident buffers,
callbacks, the key-value logger and ``model.zip`` I/O."""
