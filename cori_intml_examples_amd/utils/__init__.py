from .env import default_device, env_flag, set_random_seed
