"""ONNX layer: protobuf schema (no `onnx` package needed), exporter with contrib Rfft/Irfft
symbolics, and a graph importer/executor."""
from .exporter import (  # noqa: F401
    AMD_DOMAIN, CONTRIB_DOMAIN, Irfft, OnnxIrfft2, OnnxRfft2, Rfft, export, irfft, register_symbolic,
    register_symbolics, rfft,
)
from .proto import load_model  # noqa: F401
from .runner import OnnxGraph, register_op, supported_ops  # noqa: F401
