"""Tests use the product's synthetic-input generator (allreduce-over-mpi_amd/ftar/inputs.py),
loaded by path so that oracle-only tests do not need libftar.so."""
import importlib.util
import os
import sys

_p = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "allreduce-over-mpi_amd", "ftar", "inputs.py")
_spec = importlib.util.spec_from_file_location("ftar_inputs_impl", _p)
_m = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(_m)
sys.modules.setdefault("ftar_inputs_impl", _m)
globals().update({k: v for k, v in vars(_m).items() if not k.startswith("__")})
