"""GPU-side data pipeline pieces."""
