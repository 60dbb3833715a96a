"""MI355X-native batched straight-highway simulator (drop-in for ttrl_env's env.step() hot path)."""
__version__ = "0.1.0"
