"""Layers, aggregators, encoders, metrics, optimizers (reference tf_euler/python/utils)."""
