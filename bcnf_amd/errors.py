"""Exceptions of the training loop (reference src/bcnf/errors.py:1)."""


class TrainingDivergedError(Exception):
    """Raised when a training loss exceeds 1e5 or is NaN after epoch 10 (trainer.py:168-169)."""
