"""bgx — MI355X-native backgammon self-play engine (drop-in for the reference's
env / agent hot path)."""
from .engine import Engine, encode  # noqa: F401
