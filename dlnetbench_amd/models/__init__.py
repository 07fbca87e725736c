"""Model architectures (registry) and the roofline workload generator."""
from .registry import MODELS, ModelArch, get_model  # noqa: F401
from .roofline import DEVICES, compute_stats, write_arch_json, write_stats  # noqa: F401
