"""shredword — MI355X-native BPE trainer, drop-in for shivendrra/shredword-trainer's BPE path.

Same import surface as the reference package (reference shredword/__init__.py:1):
``from shredword.trainer import BPETrainer``.
"""
from .trainer import BPETrainer, UnigramTrainer

__version__ = "0.1.0+mi355x"
