"""Context-aware MoE FFN for RT-DETR on MI355X (HIP kernels via libmoe_hip.so)."""
from .config import MoEConfig, parse_moe_spec  # noqa: F401
from .context import CONTEXT_LABELS, NUM_CONTEXTS, solar_context_id  # noqa: F401
