from .config import TrainConfig, parse, parser
from .trainer import Trainer, run


def main(mode: str, argv=None) -> dict:
    """Entry point shared by the three reference-named scripts."""
    return run(parse(mode, argv))


__all__ = ["TrainConfig", "Trainer", "main", "parse", "parser", "run"]
