"""bhrt -- Python view of the MI355X geodesic ray tracer (libbhrt.so).

abi      ctypes mirror of the C ABI (reference types + bhrt_* extension structs)
configs  the BASELINE.json configurations C1..C5 and cameras A/B/V
lib      binding of libbhrt.so (GPU only; raises BhrtError when it cannot run)
"""
from . import abi, configs  # noqa: F401
