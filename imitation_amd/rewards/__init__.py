"""Reward models, reward-fn protocol, env reward wrappers and the reward registry."""
