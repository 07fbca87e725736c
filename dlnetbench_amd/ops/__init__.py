"""Torch-facing wrappers of the hand-written gfx950 kernels (libdlnb.so)."""
