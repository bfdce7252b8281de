from .cartpole_env import CartpoleEnv  # noqa: F401
