"""Registers blendtorch-cartpole-v0 with gym when gym is installed."""
try:
    from gym.envs.registration import register
    register(id='blendtorch-cartpole-v0', entry_point='cartpole_gym.envs:CartpoleEnv')
except ImportError:
    pass
