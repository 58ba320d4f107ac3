"""Dataset classes (reference imaginaire/datasets/*)."""
