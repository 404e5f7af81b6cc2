"""Engine layer: static-shape hipGraph engines built from ONNX or nn.Module (TensorRT-plan analogue)."""
from .engine import ENGINE_MAGIC, Binding, Engine, EngineHeader  # noqa: F401
