"""ftar — Python host binding of libftar.so (the MI355X FlexTree AllReduce).

A thin ctypes layer over the C ABI in include/ftar.h.  It mirrors the
reference's call surface (allreduce_over_mpi/mpi_mod.hpp:1723-1778):

    MPI_Allreduce_FT(sendbuf, recvbuf, count, datatype, op, comm)
        -> ftar.allreduce(sendbuf, recvbuf, count, dtype, op, comm, stream=...)

with MPI_IN_PLACE == `sendbuf=None`, MPI datatypes/ops mapped to DTYPE/OP,
and FT_TOPO / FT_LONELY read from the environment exactly like get_stages
(mpi_mod.hpp:1419-1486) — or passed explicitly as `topo="2,4"`, `lonely=1`.

Buffers are device pointers (ints) or objects with `data_ptr()` (torch
tensors).  There is no CPU fallback: if libftar.so is missing this module
raises at import time.
"""
import ctypes
import json
import os

from .names import kernel_symbol  # noqa: F401  (re-exported)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FTAR_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libftar.so"))

if not os.path.exists(LIB_PATH):
    raise ImportError(f"libftar.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                      "or `make -C allreduce-over-mpi_amd/csrc`")

# One HIP runtime per process: torch ships its own libamdhip64/librccl with the
# same sonames (libamdhip64.so.7, librccl.so.1) as the ROCm ones libftar links.
# Loading torch first makes libftar's DT_NEEDED entries bind to those copies
# instead of mapping a second runtime next to torch's.
try:
    import torch  # noqa: F401
except ImportError:  # standalone use: libftar loads /opt/rocm's runtime
    pass

_lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)

# ---- enums (include/ftar.h) -------------------------------------------------
DTYPE = {"u8": 0, "i8": 1, "u16": 2, "i16": 3, "i32": 4, "i64": 5, "f32": 6, "f64": 7, "bool": 8, "bf16": 9}
# MPI names used by the reference (mpi_mod.hpp:1365-1375)
MPI_DTYPE = {"MPI_UINT8_T": 0, "MPI_INT8_T": 1, "MPI_UINT16_T": 2, "MPI_INT16_T": 3, "MPI_INT32_T": 4,
             "MPI_INT64_T": 5, "MPI_LONG_LONG": 5, "MPI_LONG_LONG_INT": 5, "MPI_FLOAT": 6, "MPI_DOUBLE": 7,
             "MPI_C_BOOL": 8}
OP = {"sum": 0, "band": 1, "MPI_SUM": 0, "MPI_BAND": 1}
ALLGATHER = {"stages": 0, "collective": 1, "direct": 2}   # ftar_allgather_t
_AG_NAME = {v: k for k, v in ALLGATHER.items()}
REDUCE_SCATTER = {"stages": 0, "direct": 1}                 # ftar_reduce_scatter_t
_RS_NAME = {v: k for k, v in REDUCE_SCATTER.items()}
STATUS = {0: "success", 1: "invalid argument", 2: "unsupported", 3: "invalid FT_TOPO/FT_LONELY",
          4: "HIP error", 5: "RCCL error", 6: "internal error", 7: "timeout",
          8: "out of device memory"}
MAX_STAGES = 16
MAX_K = 64          # FTAR_MAX_K (ftar.h): sources of one reduce, segments of one gather
_TORCH_DTYPE_NAMES = {"torch.float32": "f32", "torch.float64": "f64", "torch.bfloat16": "bf16", "torch.int32": "i32",
                      "torch.int64": "i64", "torch.int16": "i16", "torch.int8": "i8", "torch.uint8": "u8",
                      "torch.bool": "bool", "torch.uint16": "u16"}


class FtarError(RuntimeError):
    def __init__(self, status, what=""):
        detail = _lib.ftar_last_error().decode()
        super().__init__(f"{what}: {STATUS.get(status, status)}" + (f" ({detail})" if detail else ""))
        self.status = status


class Topo(ctypes.Structure):
    _fields_ = [("nstages", ctypes.c_int), ("stages", ctypes.c_int * MAX_STAGES), ("lonely", ctypes.c_int),
                ("ring", ctypes.c_int)]

    def __str__(self):
        buf = ctypes.create_string_buffer(128)
        _lib.ftar_topo_format(ctypes.byref(self), buf, 128)
        return buf.value.decode()

    @property
    def widths(self):
        return [self.stages[i] for i in range(self.nstages)]


class CostParams(ctypes.Structure):
    """ftar_cost_params_t: the xGMI execution model's constants (include/ftar.h)."""
    _fields_ = [(n, ctypes.c_double) for n in ("alpha_us", "link_gbps", "hbm_gbps", "issue_us", "barrier_us",
                                               "peer_read_gbps", "peer_write_gbps", "copy_gbps", "coll_gbps")]

    def as_dict(self):
        return {n: getattr(self, n) for n, _ in self._fields_}


class Exec(ctypes.Structure):
    """ftar_exec_t: what the execution model chose (topology, form, piece) and its predicted seconds."""
    _fields_ = [("topo", Topo), ("form", ctypes.c_int), ("chunk_bytes", ctypes.c_size_t), ("seconds", ctypes.c_double),
                ("tied", ctypes.c_int), ("tie_broken_by", ctypes.c_int)]

    def as_dict(self):
        d = {"topology": str(self.topo), "form": FORM_NAME.get(self.form, self.form),
             "chunk_bytes": self.chunk_bytes, "predicted_ms": self.seconds * 1e3 if self.seconds >= 0 else None,
             "tied": self.tied}
        if self.tied > 1:   # the model priced several candidates alike: say which rule picked this one
            d["tie_broken_by"] = TIE_NAME.get(self.tie_broken_by, self.tie_broken_by)
        return d


FORM = {"auto": -1, "direct": 0, "stages": 1, "collective": 2, "peer-read": 3, "peer-write": 4}   # ftar_form_t
FORM_NAME = {v: k for k, v in FORM.items()}
TIE_NAME = {0: "none", 1: "stages", 2: "form", 3: "piece"}   # ftar_tie_t
CHOOSE_TOPO, CHOOSE_FORM, CHOOSE_CHUNK, CHOOSE_PEER = 1, 2, 4, 8


class UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * 128)]


_vp, _sz, _int = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
_lib.ftar_version.restype = ctypes.c_char_p
_lib.ftar_status_string.restype = ctypes.c_char_p
_lib.ftar_last_error.restype = ctypes.c_char_p
_lib.ftar_dtype_size.restype = _sz
_lib.ftar_dtype_size.argtypes = [_int]
_lib.ftar_reduce.argtypes = [ctypes.POINTER(_vp), _int, _vp, _sz, _int, _int, _vp]
_lib.ftar_reduce_nested.argtypes = [ctypes.POINTER(_vp), _int, _vp, _sz, _int, _int, ctypes.POINTER(_int), _int, _vp]
_lib.ftar_topo_parse.argtypes = [ctypes.c_char_p, ctypes.c_char_p, _int, ctypes.POINTER(Topo)]
_lib.ftar_topo_from_env.argtypes = [_int, _sz, ctypes.POINTER(Topo)]
_lib.ftar_topo_choose.argtypes = [_int, _sz, ctypes.POINTER(Topo)]
_lib.ftar_topo_candidates.argtypes = [_int, ctypes.POINTER(Topo), _int]
_lib.ftar_topo_cost.argtypes = [ctypes.POINTER(Topo), _int, _sz]
_lib.ftar_topo_cost.restype = ctypes.c_double
_lib.ftar_cost_reference.argtypes = [ctypes.POINTER(_int), _int, _int, ctypes.c_double]
_lib.ftar_cost_reference.restype = ctypes.c_double
_lib.ftar_topo_choose_reference.argtypes = [_int, ctypes.c_double, ctypes.POINTER(Topo), ctypes.POINTER(_int)]
_lib.ftar_cost_reference_candidates.argtypes = [_int, ctypes.POINTER(_int), _int, ctypes.POINTER(_int), _int]
_lib.ftar_cost_set_params.argtypes = [ctypes.c_double] * 3
_lib.ftar_cost_get_params.argtypes = [ctypes.POINTER(ctypes.c_double)] * 3
_lib.ftar_cost_set.argtypes = [ctypes.POINTER(CostParams)]
_lib.ftar_cost_get.argtypes = [ctypes.POINTER(CostParams)]
_lib.ftar_cost_load.argtypes = [ctypes.c_char_p]
_lib.ftar_cost_save.argtypes = [ctypes.c_char_p]
_lib.ftar_cost_predict.argtypes = [ctypes.POINTER(Topo), _int, _sz, _int, _sz, _int]
_lib.ftar_cost_predict.restype = ctypes.c_double
_lib.ftar_exec_choose.argtypes = [_int, _sz, _int, ctypes.POINTER(Exec)]
_lib.ftar_comm_set_form.argtypes = [_vp, _int]
_lib.ftar_comm_get_form.argtypes = [_vp, ctypes.POINTER(_int)]
_lib.ftar_comm_last_exec.argtypes = [_vp, ctypes.POINTER(Exec)]
_lib.ftar_topo_format.argtypes = [ctypes.POINTER(Topo), ctypes.c_char_p, _sz]
_lib.ftar_get_unique_id.argtypes = [ctypes.POINTER(UniqueId)]
_lib.ftar_comm_init_rank.argtypes = [ctypes.POINTER(_vp), _int, UniqueId, _int, _int]
_lib.ftar_comm_init_local.argtypes = [ctypes.POINTER(_vp), _int, ctypes.POINTER(_int)]
_lib.ftar_comm_destroy.argtypes = [_vp]
_lib.ftar_comm_set_chunk_bytes.argtypes = [_vp, _sz]
_lib.ftar_comm_get_chunk_bytes.argtypes = [_vp, ctypes.POINTER(_sz)]
_lib.ftar_allreduce.argtypes = [_vp, _vp, _sz, _int, _int, ctypes.POINTER(Topo), _vp, _vp]
_lib.ftar_rccl_allreduce.argtypes = [_vp, _vp, _sz, _int, _int, _vp, _vp]
_lib.ftar_allreduce_group.argtypes = [ctypes.POINTER(_vp), ctypes.POINTER(_vp), _sz, _int, _int, ctypes.POINTER(Topo),
                                      ctypes.POINTER(_vp), _int, ctypes.POINTER(_vp)]
_lib.ftar_allreduce_host.argtypes = [_vp, _vp, _sz, _int, _int, ctypes.POINTER(Topo), _vp, _vp]
_lib.ftar_allreduce_host_group.argtypes = [ctypes.POINTER(_vp), ctypes.POINTER(_vp), _sz, _int, _int,
                                           ctypes.POINTER(Topo), ctypes.POINTER(_vp), _int, ctypes.POINTER(_vp)]
_lib.ftar_comm_set_peer_direct.argtypes = [_vp, _int]
_lib.ftar_debug_set_peer_tuning.argtypes = [_vp, _int, _int]
_lib.ftar_debug_set_peer_dma.argtypes = [_vp, _int]
_lib.ftar_debug_set_rccl_register.argtypes = [_vp, _int]
_lib.ftar_debug_set_peer_wg_cap.argtypes = [_vp, _sz]
_lib.ftar_debug_exchange_buffer.argtypes = [_vp, _int, ctypes.POINTER(_vp), ctypes.POINTER(_sz)]
_lib.ftar_debug_gather_log.argtypes = [_vp, _sz, ctypes.POINTER(_vp), ctypes.POINTER(_vp), ctypes.POINTER(_sz)]
_lib.ftar_comm_get_peer_direct.argtypes = [_vp, ctypes.POINTER(_int)]
_lib.ftar_xgmi_probe.argtypes = [_vp, _sz, _int, ctypes.POINTER(ctypes.c_double), _int]
_lib.ftar_debug_xgmi_probe_cap.argtypes = [_vp, _sz, _int, _sz, ctypes.POINTER(ctypes.c_double), _int]
_lib.ftar_comm_set_phase_timing.argtypes = [_vp, _int]
_lib.ftar_comm_register.argtypes = [_vp, _vp, _sz, ctypes.POINTER(_int)]
_HOST_ALLGATHER = ctypes.CFUNCTYPE(_int, _vp, _vp, _sz, _vp)
_lib.ftar_comm_init_host.argtypes = [ctypes.POINTER(_vp), _int, _int, _int, _HOST_ALLGATHER, _vp]
_lib.ftar_comm_deregister.argtypes = [_vp, _int]
_lib.ftar_comm_phase_json.argtypes = [_vp, ctypes.c_char_p, _sz]
_lib.ftar_comm_phase_json.restype = ctypes.c_long
PEER_MODE = {"off": 0, "read": 1, "write": 2}                # ftar_peer_mode_t


def _peer_mode(mode):
    if isinstance(mode, str):
        return PEER_MODE[mode]
    if mode is True or mode is False:
        return int(mode)
    return int(mode)
_lib.ftar_comm_set_reduce_cus.argtypes = [_vp, _int]
_lib.ftar_comm_get_reduce_cus.argtypes = [_vp, ctypes.POINTER(_int)]
_lib.ftar_comm_set_host_chunk_bytes.argtypes = [_vp, _sz]
_lib.ftar_comm_get_host_chunk_bytes.argtypes = [_vp, ctypes.POINTER(_sz)]
_lib.ftar_schedule_json.argtypes = [ctypes.POINTER(Topo), _int, _int, _sz, ctypes.c_char_p, _sz]
_lib.ftar_schedule_json.restype = ctypes.c_long
_lib.ftar_plan_json.argtypes = [ctypes.POINTER(Topo), _int, _int, _sz, _int, _int, ctypes.c_char_p, _sz]
_lib.ftar_comm_set_reduce_scatter.argtypes = [_vp, _int]
_lib.ftar_comm_get_reduce_scatter.argtypes = [_vp, ctypes.POINTER(_int)]
_lib.ftar_comm_set_allgather.argtypes = [_vp, _int]
_lib.ftar_comm_get_allgather.argtypes = [_vp, ctypes.POINTER(_int)]
_lib.ftar_plan_json.restype = ctypes.c_long
_lib.ftar_debug_last_kernel.argtypes = [ctypes.c_char_p, _sz]
_lib.ftar_debug_last_kernel.restype = ctypes.c_long


def lib():
    return _lib


_bench_lib = None


def bench_lib():
    """libftar_bench.so: the A/B kernel variants (ftar_debug_reduce_variant, ftar_debug_reduce_nested_lds) and
    kernel test hooks (ftar_debug_bf16_cvt_check) that tools/kbench*.py and the tests load; kept out of the
    product library, which holds only the kernels the engine dispatches."""
    global _bench_lib
    if _bench_lib is None:
        _bench_lib = ctypes.CDLL(os.path.join(os.path.dirname(LIB_PATH), "libftar_bench.so"))
    return _bench_lib


def version():
    return _lib.ftar_version().decode()


def last_error():
    """ftar_last_error(): detail of the last failure on the calling thread ("" if none)."""
    return _lib.ftar_last_error().decode(errors="replace")


def _check(st, what):
    if st != 0:
        raise FtarError(st, what)


def _dt(dtype):
    if isinstance(dtype, int):
        return dtype
    s = str(dtype)
    if s in DTYPE:
        return DTYPE[s]
    if s in MPI_DTYPE:
        return MPI_DTYPE[s]
    if s in _TORCH_DTYPE_NAMES:
        return DTYPE[_TORCH_DTYPE_NAMES[s]]
    raise ValueError(f"unknown dtype {dtype!r}")


def _op(op):
    return op if isinstance(op, int) else OP[op]


def _ptr(x):
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "__array_interface__"):  # numpy (host buffers of the host-mode calls)
        return x.__array_interface__["data"][0]
    raise TypeError(f"not a buffer pointer: {type(x)}")


def _stream(s):
    if s is None:
        return None
    if isinstance(s, int):
        return s
    if hasattr(s, "cuda_stream"):
        return s.cuda_stream
    raise TypeError(f"not a stream: {type(s)}")


def dtype_size(dtype):
    return _lib.ftar_dtype_size(_dt(dtype))


def last_kernel():
    """The kernel ftar's reduce/copy launchers last launched on this thread (ftar_debug_last_kernel), as
    kernel_symbol() of its demangled name, or None."""
    n = _lib.ftar_debug_last_kernel(None, 0)
    if n < 0:
        return None
    buf = ctypes.create_string_buffer(n + 1)
    _lib.ftar_debug_last_kernel(buf, n + 1)
    return kernel_symbol(buf.value.decode())


# ---- L3: one-device reduce ----------------------------------------------------
def reduce(srcs, dst, count, dtype="f32", op="sum", stream=None, shape=None):
    """dst[i] = srcs[0][i] op srcs[1][i] op ... (left to right), enqueued on `stream`.
    shape=[w0, w1, ...]: nested fold of the sources in depth-first leaf order (ftar_reduce_nested)."""
    arr = (_vp * len(srcs))(*[_ptr(s) for s in srcs])
    if shape is None:
        _check(_lib.ftar_reduce(arr, len(srcs), _ptr(dst), count, _dt(dtype), _op(op), _stream(stream)),
               "ftar_reduce")
    else:
        sh = (_int * max(1, len(shape)))(*shape)
        _check(_lib.ftar_reduce_nested(arr, len(srcs), _ptr(dst), count, _dt(dtype), _op(op), sh, len(shape),
                                       _stream(stream)), "ftar_reduce_nested")


# ---- topology -------------------------------------------------------------------
def topo(spec=None, lonely=0, nranks=None):
    """Topo from "2,4" / [2,4] / "ring" (+ lonely count), validated for nranks if given."""
    if isinstance(spec, Topo):
        return spec
    if spec in ("ring", 1, "1"):
        spec = "1"
    if isinstance(spec, (list, tuple)):
        spec = ",".join(str(x) for x in spec)
    if nranks is None:
        t = Topo()
        ws = [int(x) for x in str(spec).split(",") if x.strip()]
        if 1 in ws:
            t.nstages, t.stages[0], t.ring = 1, 1, 1
            return t
        t.nstages = len(ws)
        for i, w in enumerate(ws):
            t.stages[i] = w
        t.lonely = int(lonely)
        return t
    t = Topo()
    _check(_lib.ftar_topo_parse(str(spec).encode(), str(lonely).encode(), nranks, ctypes.byref(t)), f"topo {spec}+{lonely}")
    return t


def topo_parse(ft_topo, ft_lonely, nranks):
    t = Topo()
    st = _lib.ftar_topo_parse(None if ft_topo is None else ft_topo.encode(),
                              None if ft_lonely is None else str(ft_lonely).encode(), nranks, ctypes.byref(t))
    _check(st, "ftar_topo_parse")
    return t


def topo_from_env(nranks, nbytes):
    t = Topo()
    _check(_lib.ftar_topo_from_env(nranks, nbytes, ctypes.byref(t)), "ftar_topo_from_env")
    return t


def topo_choose(nranks, nbytes):
    t = Topo()
    _check(_lib.ftar_topo_choose(nranks, nbytes, ctypes.byref(t)), "ftar_topo_choose")
    return t


def topo_candidates(nranks):
    n = _lib.ftar_topo_candidates(nranks, None, 0)
    if n < 0:
        raise FtarError(-n, "ftar_topo_candidates")
    arr = (Topo * max(1, n))()
    _lib.ftar_topo_candidates(nranks, arr, n)
    return [arr[i] for i in range(n)]


def topo_cost(t, nranks, nbytes):
    return _lib.ftar_topo_cost(ctypes.byref(topo(t)), nranks, nbytes)


def cost_reference(widths, nranks, chunk=100.0):
    """The reference's CostModel score of one getWidth-style width list (cost_model/CostModel.h:1-120)."""
    arr = (_int * len(widths))(*widths)
    return _lib.ftar_cost_reference(arr, len(widths), nranks, chunk)


def reference_candidates(nranks):
    """getWidth(P) (cost_model/GetWidth.h:42-47) as lists, [1,P] and [P,1] included."""
    n = _lib.ftar_cost_reference_candidates(nranks, None, 0, None, 0)
    if n < 0:
        raise FtarError(-n, "ftar_cost_reference_candidates")
    lens = (_int * n)()
    _lib.ftar_cost_reference_candidates(nranks, None, 0, lens, n)
    tot = sum(lens)
    ws = (_int * tot)()
    _lib.ftar_cost_reference_candidates(nranks, ws, tot, lens, n)
    out, at = [], 0
    for ln in lens:
        out.append(list(ws[at:at + ln]))
        at += ln
    return out


def topo_choose_reference(nranks, chunk=100.0):
    """The reference cost model's argmin (CostModel.h:82-120): (topology, index into reference_candidates)."""
    t, i = Topo(), _int(0)
    _check(_lib.ftar_topo_choose_reference(nranks, chunk, ctypes.byref(t), ctypes.byref(i)),
           "ftar_topo_choose_reference")
    return t, i.value


def cost_params(alpha_us=None, link_gbps=None, hbm_gbps=None):
    """Read, or set (process-wide; 0 restores the default), the xGMI cost model's constants."""
    if alpha_us is not None or link_gbps is not None or hbm_gbps is not None:
        _check(_lib.ftar_cost_set_params(alpha_us or 0.0, link_gbps or 0.0, hbm_gbps or 0.0), "ftar_cost_set_params")
    v = [ctypes.c_double() for _ in range(3)]
    _check(_lib.ftar_cost_get_params(*[ctypes.byref(x) for x in v]), "ftar_cost_get_params")
    return {"alpha_us": v[0].value, "link_GBps": v[1].value, "hbm_GBps": v[2].value}


def cost_get():
    """Every constant of the xGMI execution model (defaults <- cost_set <- FTAR_COST_* environment)."""
    p = CostParams()
    _check(_lib.ftar_cost_get(ctypes.byref(p)), "ftar_cost_get")
    return p.as_dict()


def cost_set(**kw):
    """Set the execution model's constants (process-wide); names as in cost_get(); a field left out or <= 0
    keeps (or restores) its default.  Returns cost_get()."""
    p = CostParams(**{k: float(v or 0.0) for k, v in kw.items()})
    _check(_lib.ftar_cost_set(ctypes.byref(p)), "ftar_cost_set")
    return cost_get()


def cost_load(path):
    """Load the execution model's constants from a calibration file (ftar_cost_load; FTAR_COST_FILE does the
    same at first use, and takes precedence); None forgets the loaded ones.  Returns cost_get()."""
    _check(_lib.ftar_cost_load(None if path is None else os.fsencode(path)), "ftar_cost_load")
    return cost_get()


def cost_save(path):
    """Write the constants in effect to a calibration file (ftar_cost_save)."""
    _check(_lib.ftar_cost_save(os.fsencode(path)), "ftar_cost_save")


def cost_predict(t, form, chunk_bytes, nranks, nbytes, registered=False):
    """Predicted seconds of one AllReduce (ftar_cost_predict); None where it cannot run that way."""
    v = _lib.ftar_cost_predict(ctypes.byref(topo(t)), FORM[form] if isinstance(form, str) else form, chunk_bytes,
                               nranks, nbytes, int(registered))
    return None if v < 0 else v


def exec_choose(nranks, nbytes, topo_=None, form=None, chunk_bytes=None, peer=True):
    """The execution model's choice (ftar_exec_choose): whatever is None is chosen; returns an Exec."""
    e = Exec()
    flags = 0
    if topo_ is None:
        flags |= CHOOSE_TOPO
    else:
        e.topo = topo(topo_)
    if form is None:
        flags |= CHOOSE_FORM | (CHOOSE_PEER if peer else 0)
    else:
        e.form = FORM[form] if isinstance(form, str) else form
    if chunk_bytes is None:
        flags |= CHOOSE_CHUNK
    else:
        e.chunk_bytes = chunk_bytes
    _check(_lib.ftar_exec_choose(nranks, nbytes, flags, ctypes.byref(e)), "ftar_exec_choose")
    return e


def schedule_json(t, nranks, rank, count):
    t = topo(t)
    n = _lib.ftar_schedule_json(ctypes.byref(t), nranks, rank, count, None, 0)
    if n < 0:
        raise FtarError(-n, "ftar_schedule_json")
    buf = ctypes.create_string_buffer(n + 1)
    _lib.ftar_schedule_json(ctypes.byref(t), nranks, rank, count, buf, n + 1)
    return json.loads(buf.value.decode())


def plan_json(t, nranks, rank, count, allgather="direct", reduce_scatter="direct"):
    t = topo(t)
    ag = ALLGATHER[allgather] if isinstance(allgather, str) else int(allgather)
    rs = REDUCE_SCATTER[reduce_scatter] if isinstance(reduce_scatter, str) else int(reduce_scatter)
    n = _lib.ftar_plan_json(ctypes.byref(t), nranks, rank, count, ag, rs, None, 0)
    if n < 0:
        raise FtarError(-n, "ftar_plan_json")
    buf = ctypes.create_string_buffer(n + 1)
    _lib.ftar_plan_json(ctypes.byref(t), nranks, rank, count, ag, rs, buf, n + 1)
    return json.loads(buf.value.decode())


# ---- communicators -------------------------------------------------------------
def get_unique_id():
    u = UniqueId()
    _check(_lib.ftar_get_unique_id(ctypes.byref(u)), "ftar_get_unique_id")
    return ctypes.string_at(ctypes.addressof(u), 128)


class Comm:
    """One rank's communicator (RCCL over xGMI, or a rank of a local group)."""

    def __init__(self, handle, rank, nranks, device, group=None):
        self.handle, self.rank, self.nranks, self.device, self._group = handle, rank, nranks, device, group

    @classmethod
    def init_rank(cls, nranks, unique_id, rank, device):
        u = UniqueId()
        ctypes.memmove(ctypes.addressof(u), unique_id, 128)
        h = _vp()
        _check(_lib.ftar_comm_init_rank(ctypes.byref(h), nranks, u, rank, device), "ftar_comm_init_rank")
        return cls(h.value, rank, nranks, device)

    @classmethod
    def init_host(cls, nranks, rank, device, allgather):
        """One process per rank, bootstrapped by the caller's host collective (ftar_comm_init_host):
        allgather(mine: bytes) -> list of every rank's bytes.  Peer-direct forms only."""
        def cb(mine, all_, nbytes, user):
            try:
                parts = allgather(ctypes.string_at(mine, nbytes))
                for r, b in enumerate(parts):
                    ctypes.memmove(all_ + r * nbytes, b, nbytes)
                return 0
            except Exception:  # noqa: BLE001  reported to the library as a failed collective
                return 1
        fn = _HOST_ALLGATHER(cb)
        h = _vp()
        _check(_lib.ftar_comm_init_host(ctypes.byref(h), nranks, rank, device, fn, None), "ftar_comm_init_host")
        c = cls(h.value, rank, nranks, device)
        c._host_cb = fn   # the library calls it for as long as the communicator lives
        return c

    @classmethod
    def init_local(cls, nranks, devices=None):
        hs = (_vp * nranks)()
        devs = (_int * nranks)(*(devices or [0] * nranks))
        _check(_lib.ftar_comm_init_local(hs, nranks, devs), "ftar_comm_init_local")
        comms = [cls(hs[r], r, nranks, devs[r]) for r in range(nranks)]
        group = LocalGroup(comms)
        for c in comms:
            c._group = group
        return group

    @property
    def chunk_bytes(self):
        v = _sz()
        _check(_lib.ftar_comm_get_chunk_bytes(self.handle, ctypes.byref(v)), "chunk_bytes")
        return v.value

    @chunk_bytes.setter
    def chunk_bytes(self, b):
        _check(_lib.ftar_comm_set_chunk_bytes(self.handle, b), "chunk_bytes")

    @property
    def form(self):
        """The data-movement form: "auto" (the execution model chooses per call), a form name, or -2 (a mix of
        all-gather / reduce-scatter settings no form names)."""
        v = _int()
        _check(_lib.ftar_comm_get_form(self.handle, ctypes.byref(v)), "form")
        return FORM_NAME.get(v.value, v.value)

    @form.setter
    def form(self, f):
        _check(_lib.ftar_comm_set_form(self.handle, FORM[f] if isinstance(f, str) else f), "form")

    def last_exec(self):
        """What the last call on this communicator ran (ftar_comm_last_exec), as a dict."""
        e = Exec()
        _check(_lib.ftar_comm_last_exec(self.handle, ctypes.byref(e)), "last_exec")
        return e.as_dict()

    def allreduce(self, sendbuf, recvbuf, count, dtype="f32", op="sum", topo_=None, lonely=0, stream=None):
        t = None if topo_ is None else ctypes.byref(topo(topo_, lonely))
        st = _lib.ftar_allreduce(_ptr(sendbuf), _ptr(recvbuf), count, _dt(dtype), _op(op), t, self.handle,
                                 _stream(stream))
        _check(st, "ftar_allreduce")

    def allreduce_host(self, sendbuf, recvbuf, count, dtype="f32", op="sum", topo_=None, lonely=0, stream=None):
        """AllReduce of HOST buffers (pinned for overlap), H2D/exchange/D2H pipelined (ftar_allreduce_host)."""
        t = None if topo_ is None else ctypes.byref(topo(topo_, lonely))
        st = _lib.ftar_allreduce_host(_ptr(sendbuf), _ptr(recvbuf), count, _dt(dtype), _op(op), t, self.handle,
                                      _stream(stream))
        _check(st, "ftar_allreduce_host")

    @property
    def peer_direct(self):
        """Peer-direct data movement for one-round plans (IPC-mapped exchange buffers, no RCCL data path):
        0 off, 1 read (folds and the all-gather pull from peers), 2 write (peers' blocks are pushed)."""
        v = _int()
        _check(_lib.ftar_comm_get_peer_direct(self.handle, ctypes.byref(v)), "peer_direct")
        return v.value

    @peer_direct.setter
    def peer_direct(self, mode):
        _check(_lib.ftar_comm_set_peer_direct(self.handle, _peer_mode(mode)), "peer_direct")

    @property
    def rccl_register(self):
        return getattr(self, "_rccl_register", False)

    @rccl_register.setter
    def rccl_register(self, on):
        """RCCL registration (ncclCommRegister) of the comm's scratch buffer (FTAR_RCCL_REGISTER); buffers
        passed to register() are always registered with RCCL too, where RCCL accepts them."""
        _check(_lib.ftar_debug_set_rccl_register(self.handle, 1 if on else 0), "rccl_register")
        self._rccl_register = bool(on)

    @property
    def peer_wg_cap(self):
        return getattr(self, "_peer_wg_cap", 0)

    @peer_wg_cap.setter
    def peer_wg_cap(self, n):
        """Workgroups per segment of the peer forms' cross-GPU copies (0 = as many as a segment fills)."""
        _check(_lib.ftar_debug_set_peer_wg_cap(self.handle, int(n)), "peer_wg_cap")
        self._peer_wg_cap = int(n)

    def peer_tuning(self, nt=True, lds=True, dma=False):
        """Peer forms: nontemporal copies (nt), the LDS-staged fold (lds; False = register kernel), and the
        cross-GPU copies by the DMA engines (dma).  Tuning hook for bench.py's sweep
        (ftar_debug_set_peer_tuning / _dma); results are identical either way."""
        _check(_lib.ftar_debug_set_peer_tuning(self.handle, 1 if nt else 0, 1 if lds else 0), "peer_tuning")
        _check(_lib.ftar_debug_set_peer_dma(self.handle, 1 if dma else 0), "peer_dma")

    def register(self, buf, nbytes):
        """Collective: register this rank's buffer (device pointer or tensor) for the peer forms' in-place
        paths (ftar_comm_register); returns the registration id (the same on every rank)."""
        r = _int()
        _check(_lib.ftar_comm_register(self.handle, _ptr(buf), nbytes, ctypes.byref(r)), "ftar_comm_register")
        return r.value

    def deregister(self, reg):
        _check(_lib.ftar_comm_deregister(self.handle, reg), "ftar_comm_deregister")

    def phase_timing(self, on=True):
        """Record timing events at the phase boundaries of every following call (diagnostic)."""
        _check(_lib.ftar_comm_set_phase_timing(self.handle, 1 if on else 0), "phase_timing")

    def last_phases(self):
        """[(phase, ms since the call's start), ...] of the last call made with phase timing on (waits for it)."""
        n = _lib.ftar_comm_phase_json(self.handle, None, 0)
        if n < 0:
            raise FtarError(-n, "ftar_comm_phase_json")
        buf = ctypes.create_string_buffer(n + 1)
        _lib.ftar_comm_phase_json(self.handle, buf, n + 1)
        return [tuple(p) for p in json.loads(buf.value.decode())]

    def xgmi_probe(self, bytes_per_peer=64 << 20, iters=10, wg_per_peer=0):
        """Collective xGMI calibration (ftar_xgmi_probe): GB/s of copy kernels through the exchange buffers,
        every rank running the same pattern at once.  wg_per_peer > 0 caps the copy kernel at that many
        256-thread workgroups per peer (how many CUs it takes to fill the links)."""
        k = 5 if wg_per_peer else 7   # (the DMA modes do not depend on a workgroup cap)
        out = (ctypes.c_double * k)()
        if wg_per_peer:
            _check(_lib.ftar_debug_xgmi_probe_cap(self.handle, bytes_per_peer, iters, wg_per_peer, out, k),
                   "ftar_debug_xgmi_probe_cap")
        else:
            _check(_lib.ftar_xgmi_probe(self.handle, bytes_per_peer, iters, out, k), "ftar_xgmi_probe")
        return dict(zip(("local_copy", "read_one_peer", "read_all_peers", "write_one_peer", "write_all_peers",
                         "dma_read_all_peers", "dma_write_all_peers"), (round(v, 2) for v in out)))

    def exchange_buffer(self, peer):
        """Test hook (ftar_debug_exchange_buffer): (device pointer, bytes) of rank `peer`'s exchange buffer as
        this process maps it (peer == this rank: its own); (0, 0) before the first peer-form call."""
        p, n = _vp(), _sz()
        _check(_lib.ftar_debug_exchange_buffer(self.handle, int(peer), ctypes.byref(p), ctypes.byref(n)),
               "exchange_buffer")
        return (p.value or 0), n.value

    def gather_log(self, piece):
        """Test hook (ftar_debug_gather_log): the gather records of piece `piece` of the last host
        call made under FTAR_DEBUG_HOST_GATHER_LOG=1, or None past the pieces logged.  A dict: pieces (logged),
        grid, nsegs, tile_bytes, off / bytes (each segment's destination in the exchange buffer), host (a
        numpy uint32 [grid, 4]: 0x80000000 | XCD, HW_ID, wall clock at start, at end; all 0 if the workgroup
        left no record) and dev_ptr (device address of grid x 2 uint32 words: how many times each workgroup id ran,
        and the XCDs it ran on as a bit set)."""
        import numpy as np
        h, d = _vp(), _vp()
        info = (_sz * (4 + 2 * MAX_K))()
        _check(_lib.ftar_debug_gather_log(self.handle, int(piece), ctypes.byref(h), ctypes.byref(d), info),
               "gather_log")
        if not h.value:
            return None
        grid, nsegs = int(info[1]), int(info[2])
        host = np.frombuffer(ctypes.string_at(h.value, grid * 16), dtype=np.uint32).reshape(grid, 4).copy()
        return {"pieces": int(info[0]), "grid": grid, "nsegs": nsegs, "tile_bytes": int(info[3]),
                "off": [int(info[4 + j]) for j in range(nsegs)],
                "bytes": [int(info[4 + MAX_K + j]) for j in range(nsegs)], "host": host, "dev_ptr": d.value}

    @property
    def reduce_cus(self):
        """CUs the reduce stream may use (0 = all): leaves the rest to the transport's kernels."""
        v = _int()
        _check(_lib.ftar_comm_get_reduce_cus(self.handle, ctypes.byref(v)), "reduce_cus")
        return v.value

    @reduce_cus.setter
    def reduce_cus(self, n):
        _check(_lib.ftar_comm_set_reduce_cus(self.handle, int(n)), "reduce_cus")

    @property
    def host_chunk_bytes(self):
        v = _sz()
        _check(_lib.ftar_comm_get_host_chunk_bytes(self.handle, ctypes.byref(v)), "host_chunk_bytes")
        return v.value

    @host_chunk_bytes.setter
    def host_chunk_bytes(self, b):
        _check(_lib.ftar_comm_set_host_chunk_bytes(self.handle, b), "host_chunk_bytes")

    @property
    def allgather(self):
        """All-gather form: "direct" (default), "stages" (the reference's rounds) or "collective"."""
        v = _int()
        _check(_lib.ftar_comm_get_allgather(self.handle, ctypes.byref(v)), "allgather")
        return _AG_NAME[v.value]

    @allgather.setter
    def allgather(self, mode):
        _check(_lib.ftar_comm_set_allgather(self.handle, ALLGATHER[mode] if isinstance(mode, str) else int(mode)),
               "allgather")

    @property
    def reduce_scatter(self):
        """Reduce-scatter form of the ring and of multi-stage trees: "direct" (one all-links round, default) or
        "stages" (the reference's)."""
        v = _int()
        _check(_lib.ftar_comm_get_reduce_scatter(self.handle, ctypes.byref(v)), "reduce_scatter")
        return _RS_NAME[v.value]

    @reduce_scatter.setter
    def reduce_scatter(self, mode):
        _check(_lib.ftar_comm_set_reduce_scatter(
            self.handle, REDUCE_SCATTER[mode] if isinstance(mode, str) else int(mode)), "reduce_scatter")

    def allreduce_tensor(self, tensor, out=None, op="sum", topo_=None, lonely=0, stream=None):
        """In-place (out=None) or out-of-place AllReduce of a contiguous device tensor,
        e.g. a data-parallel gradient bucket; dtype and count come from the tensor."""
        if not tensor.is_contiguous() or (out is not None and not out.is_contiguous()):
            raise ValueError("ftar needs contiguous tensors")
        if out is not None and (out.numel() != tensor.numel() or out.dtype != tensor.dtype):
            raise ValueError("out must match tensor in size and dtype")
        dt = _dt(str(tensor.dtype))
        if out is None:
            self.allreduce(None, tensor, tensor.numel(), dt, op, topo_, lonely, stream)
            return tensor
        self.allreduce(tensor, out, tensor.numel(), dt, op, topo_, lonely, stream)
        return out

    def rccl_allreduce(self, sendbuf, recvbuf, count, dtype="f32", op="sum", stream=None):
        """RCCL's own ncclAllReduce on this communicator (comparison yardstick)."""
        st = _lib.ftar_rccl_allreduce(_ptr(sendbuf), _ptr(recvbuf), count, _dt(dtype), _op(op), self.handle,
                                      _stream(stream))
        _check(st, "ftar_rccl_allreduce")

    def destroy(self):
        if self.handle:
            _check(_lib.ftar_comm_destroy(self.handle), "ftar_comm_destroy")
            self.handle = None


class LocalGroup:
    """All ranks of an in-process group (ftar_comm_init_local)."""

    def __init__(self, comms):
        self.comms = comms

    def __len__(self):
        return len(self.comms)

    def __getitem__(self, i):
        return self.comms[i]

    def set_chunk_bytes(self, b):
        for c in self.comms:
            c.chunk_bytes = b

    def set_form(self, f):
        for c in self.comms:
            c.form = f

    def set_allgather(self, mode):
        for c in self.comms:
            c.allgather = mode

    def set_host_chunk_bytes(self, b):
        for c in self.comms:
            c.host_chunk_bytes = b

    def set_peer_direct(self, on):
        for c in self.comms:
            c.peer_direct = on

    def set_reduce_scatter(self, mode):
        for c in self.comms:
            c.reduce_scatter = mode

    def set_reduce_cus(self, n):
        for c in self.comms:
            c.reduce_cus = n

    def register(self, bufs, nbytes):
        """Register one buffer per rank (collective: one host thread per rank); returns the ids."""
        import threading
        ids, errs = [None] * len(self.comms), []

        def run(r):
            try:
                ids[r] = self.comms[r].register(bufs[r], nbytes)
            except Exception as e:  # noqa: BLE001
                errs.append(e)
        th = [threading.Thread(target=run, args=(r,)) for r in range(len(self.comms))]
        for t in th:
            t.start()
        for t in th:
            t.join()
        if errs:
            raise errs[0]
        return ids

    def deregister(self, ids):
        for c, i in zip(self.comms, ids):
            c.deregister(i)

    def allreduce(self, sendbufs, recvbufs, count, dtype="f32", op="sum", topo_=None, lonely=0, streams=None,
                  host=False):
        """Every rank at once, enqueued on each rank's stream (None: the NULL stream), returning once enqueued;
        host=True: the buffers are host memory (ftar_allreduce_host_group), returning once they hold the result."""
        P = len(self.comms)
        t = None if topo_ is None else ctypes.byref(topo(topo_, lonely))
        sb = None if sendbufs is None else (_vp * P)(*[_ptr(x) for x in sendbufs])
        rb = (_vp * P)(*[_ptr(x) for x in recvbufs])
        hs = (_vp * P)(*[c.handle for c in self.comms])
        ss = None if streams is None else (_vp * P)(*[_stream(s) for s in streams])
        fn = _lib.ftar_allreduce_host_group if host else _lib.ftar_allreduce_group
        st = fn(sb, rb, count, _dt(dtype), _op(op), t, hs, P, ss)
        _check(st, "ftar_allreduce_host_group" if host else "ftar_allreduce_group")

    def allreduce_tensors(self, tensors, op="sum", topo_=None, lonely=0):
        """In-place AllReduce of one contiguous device tensor per rank (same shape and dtype)."""
        t0 = tensors[0]
        if any(not t.is_contiguous() or t.numel() != t0.numel() or t.dtype != t0.dtype for t in tensors):
            raise ValueError("tensors must be contiguous and alike")
        self.allreduce(None, tensors, t0.numel(), _dt(str(t0.dtype)), op, topo_, lonely)
        return tensors

    def destroy(self):
        for c in self.comms:
            c.destroy()


# ---- the reference's call surface ---------------------------------------------
MPI_IN_PLACE = None


def MPI_Allreduce_FT(sendbuf, recvbuf, count, datatype, op, comm, stream=None):
    """Drop-in for MPI_Allreduce_FT (mpi_mod.hpp:1724) on device buffers.

    sendbuf=MPI_IN_PLACE (None) reduces recvbuf in place; datatype/op accept the
    reference's MPI names ("MPI_FLOAT", "MPI_SUM"); the topology comes from
    FT_TOPO/FT_LONELY read at this call, as get_stages is (mpi_mod.hpp:1732;
    both unset: the cost model).  Returns 0 like the reference; raises
    FtarError where the reference would exit(1) (an invalid FT_TOPO among them).
    """
    comm.allreduce(sendbuf, recvbuf, count, datatype, op, stream=stream)
    return 0
