from ._secagg_utils import divide, multiply, quantize, reverse_quantize

__all__ = ["quantize", "reverse_quantize", "multiply", "divide"]
