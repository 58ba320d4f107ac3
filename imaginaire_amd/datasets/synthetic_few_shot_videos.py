"""Synthetic few-shot paired-video dataset (see datasets/synthetic.py)."""
from imaginaire_amd.datasets.synthetic import Dataset  # noqa: F401
