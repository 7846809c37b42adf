"""Training step on the HIP path (reference train/train_imc.py)."""
