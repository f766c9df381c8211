"""vitdec -- Python binding of the MI355X Viterbi decoder's C-ABI (include/vd_capi.h).

Mirrors the reference's decoder interface `ViterbiCUDA<options>` (src/viterbi/viterbi.h:43-152):
the same option bitmask, the same constexpr members (constLen, polyn1, polyn2, extraL, extraR,
bitsPerPack, encDataPerPack, ...), the same size helpers and the same `run(input, output, inputNum)`
call returning the kernel time in ms.  Errors raise VitdecError (the reference exits the process,
gpuerrors.h:8-17; the C++ header include/viterbi.h keeps that behaviour).

Device-side entry points (`run_device`, `simulate_device`) take raw device pointers, e.g.
`tensor.data_ptr()` of a torch tensor on the decoder's device, and a HIP stream handle
(`torch.cuda.current_stream().cuda_stream`).  torch is only plumbing for memory and streams.

There is no CPU fallback: if lib/libvitdec.so is missing or no GPU is visible, decoding raises.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# VITDEC_LIB (tests only): another build of the same C-ABI, e.g. the deliberately broken scratch build
# tests/test_gpu_guard.py uses to show the LDS guard check catches a real bug
LIB_PATH = os.environ.get("VITDEC_LIB") or os.path.join(_HERE, "lib", "libvitdec.so")

# ---- option bitmask (reference src/viterbi/viterbi.h:7-20) ----
CHANNEL_MASK, METRIC_MASK, DECODE_MASK, COMP_MASK = 0xF, 0xF0, 0xF00, 0xF000
HARD, SOFT4, SOFT8, SOFT16, FP32 = 0x0, 0x1, 0x2, 0x3, 0x4
M_B32, M_B16, M_FP16 = 0x00, 0x10, 0x20
O_B32, O_B16 = 0x000, 0x100
REG, DPX = 0x0000, 0x1000

INPUT_NAMES = {"HARD": HARD, "h": HARD, "SOFT4": SOFT4, "s4": SOFT4, "SOFT8": SOFT8, "s8": SOFT8,
               "SOFT16": SOFT16, "s16": SOFT16, "FP32": FP32, "f": FP32}
METRIC_NAMES = {"b16": M_B16, "b32": M_B32, "f16": M_FP16}
OUTPUT_NAMES = {"b16": O_B16, "b32": O_B32}
COMP_NAMES = {"REG": REG, "reg": REG, "DPX": DPX, "dpx": DPX}

VD_OK = 0
_ERRNAMES = {-1: "VD_ERR_OPTIONS", -2: "VD_ERR_ARG", -3: "VD_ERR_DEVICE", -4: "VD_ERR_NOMEM",
             -5: "VD_ERR_NOKERNEL"}

# every entry point declared in include/vd_capi.h (tests check the library exports all of them)
EXPORTS = ["vd_options_valid", "vd_input_size", "vd_message_len", "vd_output_size", "vd_num_chunks",
           "vd_create", "vd_destroy", "vd_run", "vd_run_device", "vd_run_device_batch", "vd_run_batches",
           "vd_simulate_host", "vd_count_errors", "vd_last_error", "vd_device_count", "vd_kernel_name",
           "vd_pack_device", "vd_run_device_llr", "vd_run_llr", "vd_host_alloc", "vd_host_free",
           "vd_run_stream", "vd_channel_device", "vd_simulate_device", "vd_mt_state_after", "vd_split_redecodes",
           "vd_split_cap_exits", "vd_set_guard_check", "vd_guard_violations", "vd_run_device_llr_batch", "vd_build_info",
           "vd_decoder_kernel_name"]


class VitdecError(RuntimeError):
    pass


_lib = None


def lib():
    """Load lib/libvitdec.so (raises if the HIP extension has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise VitdecError(f"{LIB_PATH} not built: run `make -C {_HERE}` (or __graft_entry__.build())")
    L = ctypes.CDLL(LIB_PATH)
    if not os.environ.get("VITDEC_LIB"):  # the product library must be built from the sources in this tree
        if not hasattr(L, "vd_build_info"):
            raise VitdecError(f"{LIB_PATH} predates the build record (no vd_build_info): rebuild it with "
                              f"`make -C {_HERE}`")
        L.vd_build_info.restype = ctypes.c_char_p
        stale = build_mismatch(L.vd_build_info().decode())
        if stale:
            raise VitdecError(f"{LIB_PATH} is stale ({stale}): rebuild it with `make -C {_HERE}`")
    sz, vp, i, f = ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int, ctypes.c_float
    # name: (argtypes, restype or None)
    sig = {"vd_options_valid": ([i], None),
           "vd_input_size": ([i, sz], sz), "vd_message_len": ([i, sz], sz), "vd_output_size": ([i, sz], sz),
           "vd_create": ([i, sz, i, ctypes.POINTER(vp)], None), "vd_destroy": ([vp], None),
           "vd_run": ([vp, vp, vp, sz, ctypes.POINTER(f)], None), "vd_run_device": ([vp, vp, vp, sz, vp], None),
           "vd_run_device_batch": ([vp, vp, sz, vp, sz, sz, ctypes.c_int, vp], None),
           "vd_run_batches": ([i, ctypes.POINTER(vp), ctypes.POINTER(vp), sz, i, ctypes.POINTER(i), i,
                               ctypes.POINTER(f)], None),
           "vd_simulate_host": ([i, sz, f, ctypes.c_uint32, ctypes.c_uint32, vp, vp], None),
           "vd_channel_device": ([sz, f, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp], None),
           "vd_simulate_device": ([i, sz, f, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp], None),
           "vd_mt_state_after": ([ctypes.c_uint32, ctypes.c_uint64, vp], None),
           "vd_split_redecodes": ([i, ctypes.POINTER(ctypes.c_uint64)], None),
           "vd_split_cap_exits": ([i, ctypes.POINTER(ctypes.c_uint64)], None),
           "vd_set_guard_check": ([vp, i], None), "vd_guard_violations": ([vp, ctypes.POINTER(ctypes.c_uint64)], None),
           "vd_count_errors": ([i, vp, sz, vp, sz], ctypes.c_longlong), "vd_last_error": (None, ctypes.c_char_p),
           "vd_pack_device": ([i, vp, sz, f, vp, vp], None), "vd_host_alloc": ([sz], vp), "vd_host_free": ([vp], None),
           "vd_run_stream": ([vp, ctypes.POINTER(vp), ctypes.POINTER(vp), i, sz, ctypes.POINTER(f)], None),
           "vd_run_device_llr": ([vp, vp, vp, sz, f, vp], None),
           "vd_run_llr": ([vp, vp, vp, sz, f, ctypes.POINTER(f)], None),
           "vd_run_device_llr_batch": ([vp, vp, sz, vp, sz, sz, f, ctypes.c_int, vp], None),
           "vd_kernel_name": ([i], ctypes.c_char_p),
           "vd_decoder_kernel_name": ([vp, sz, i, i], ctypes.c_char_p)}
    for name, (args, res) in sig.items():
        if not hasattr(L, name):
            if os.environ.get("VITDEC_LIB"):  # an earlier round's build in a same-box A/B: fewer entry points
                continue
            raise VitdecError(f"{LIB_PATH} does not export {name}")
        fn = getattr(L, name)
        if args is not None:
            fn.argtypes = args
        if res is not None:
            fn.restype = res
    _lib = L
    return L


def build_mismatch(info):
    """None when the sources named in the library's build record hash to the recorded value, else why not."""
    import hashlib
    parts = info.split()
    if len(parts) < 2:
        return "no build record"
    h = hashlib.sha256()
    for rel in parts[1:]:
        p = os.path.join(_HERE, rel)
        if not os.path.exists(p):
            return f"source {rel} missing"
        with open(p, "rb") as fh:
            h.update(fh.read())
    return None if h.hexdigest()[:16] == parts[0] else "sources changed since the build"


def _check(rc):
    if rc != VD_OK:
        msg = lib().vd_last_error().decode(errors="replace")
        raise VitdecError(f"{_ERRNAMES.get(rc, rc)}: {msg}")


def parse_options(input="HARD", metric="b32", output="b32", comp="REG"):
    """CLI-style names (reference src/main.cpp:174-264) -> options bitmask."""
    return INPUT_NAMES[input] | METRIC_NAMES[metric] | OUTPUT_NAMES[output] | COMP_NAMES[comp]


def options_valid(options):
    return bool(lib().vd_options_valid(options))


def device_count():
    return lib().vd_device_count()


def kernel_name(options):
    return lib().vd_kernel_name(options).decode()


class ViterbiCUDA:
    """The reference's ViterbiCUDA<options> (viterbi.h:43-152) over the C-ABI."""

    constLen = 7
    polyn1 = 0o171
    polyn2 = 0o133
    extraL_raw = extraR_raw = slideSize_raw = 32
    bmMemWidth = 32
    blockDimY = 2
    FPprecision = 4

    def __init__(self, options, inputNum=0, device=0):
        if not options_valid(options):
            raise VitdecError(f"options 0x{options:x} disabled by OptionsValid")
        self.options = options
        self.inputType = options & CHANNEL_MASK
        self.metricType = options & METRIC_MASK
        self.outputType = options & DECODE_MASK
        self.compMode = options & COMP_MASK
        self.bitsPerMetric = {M_B16: 16, M_B32: 32}.get(self.metricType, 11)
        self.bitsPerPack = 16 if self.outputType == O_B16 else 32
        rnd = lambda a, b: (a + b - 1) // b * b
        self.extraL = rnd(32, self.bitsPerPack) - (self.constLen - 1)
        self.extraR = rnd(32, self.bitsPerPack) + (self.constLen - 1)
        self.slideSize = rnd(32, self.bitsPerPack)
        self.forwardLen = self.extraL + self.slideSize + self.extraR
        self.encDataPerPack = {HARD: 32, SOFT4: 8, SOFT8: 4, SOFT16: 2, FP32: 1}[self.inputType]
        self.encDataWidth = {HARD: 1, SOFT4: 4, SOFT8: 8, SOFT16: 16, FP32: self.FPprecision}[self.inputType]
        self.encPack_t = np.float32 if self.inputType == FP32 else np.int32
        self.decPack_t = np.uint16 if self.outputType == O_B16 else np.uint32
        self.device = device
        h = ctypes.c_void_p()
        _check(lib().vd_create(options, inputNum, device, ctypes.byref(h)))
        self._h = h

    def close(self):
        if getattr(self, "_h", None):
            lib().vd_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # size helpers (viterbi.cu:63-92)
    def getInputSize(self, inputNum):
        return lib().vd_input_size(self.options, inputNum)

    def getMessageLen(self, inputNum):
        return lib().vd_message_len(self.options, inputNum)

    def getOutputSize(self, inputNum):
        return lib().vd_output_size(self.options, inputNum)

    def run(self, input_h, output_h=None, inputNum=None):
        """Blocking host decode (viterbi.cu:210-238). Returns (output array, kernel ms)."""
        input_h = np.ascontiguousarray(input_h)
        if inputNum is None:
            inputNum = input_h.size * self.encDataPerPack
        if input_h.nbytes < self.getInputSize(inputNum):
            raise VitdecError("input buffer smaller than getInputSize(inputNum)")
        if output_h is None:
            output_h = np.zeros(self.getOutputSize(inputNum) // np.dtype(self.decPack_t).itemsize,
                                dtype=self.decPack_t)
        if output_h.nbytes < self.getOutputSize(inputNum):
            raise VitdecError("output buffer smaller than getOutputSize(inputNum)")
        ms = ctypes.c_float(0.0)
        _check(lib().vd_run(self._h, input_h.ctypes.data, output_h.ctypes.data, inputNum, ctypes.byref(ms)))
        return output_h, ms.value

    def run_device(self, input_ptr, output_ptr, inputNum, stream=0):
        """Async device decode: raw device pointers on self.device, HIP stream handle (int)."""
        _check(lib().vd_run_device(self._h, ctypes.c_void_p(input_ptr), ctypes.c_void_p(output_ptr), inputNum,
                                   ctypes.c_void_p(stream)))

    def run_device_batch(self, input_ptr, input_stride, output_ptr, output_stride, inputNum, nbatch, stream=0):
        """nbatch independent batches in one launch: batch b at input_ptr + b * input_stride bytes (0: the
        same input each time) -> output_ptr + b * output_stride bytes (vd_run_device_batch)."""
        _check(lib().vd_run_device_batch(self._h, ctypes.c_void_p(input_ptr), input_stride, ctypes.c_void_p(output_ptr),
                                         output_stride, inputNum, nbatch, ctypes.c_void_p(stream)))

    def kernel_for(self, inputNum, nbatch=1, llr=False):
        """the kernel and launch form this decoder runs for nbatch batches of inputNum values
        (vd_decoder_kernel_name: follows VD_NO_PK / VD_PK_SPLIT / VD_NO_SPLIT as read at creation)"""
        return lib().vd_decoder_kernel_name(self._h, inputNum, nbatch, 1 if llr else 0).decode()

    def set_guard_check(self, enable=True):
        """LDS guard words around every wave's table and ring, counted at kernel exit when overwritten
        (vd_set_guard_check; the count restarts at 0)."""
        _check(lib().vd_set_guard_check(self._h, 1 if enable else 0))

    def guard_violations(self):
        """guard words found overwritten since set_guard_check(True) (synchronises the device)"""
        v = ctypes.c_uint64(0)
        _check(lib().vd_guard_violations(self._h, ctypes.byref(v)))
        return v.value

    def run_stream(self, inputs, inputNum=None, outputs=None):
        """Pipelined decode of independent batches (host copies overlapped with decoding).
        Returns (list of outputs, wall ms).  Pass PinnedArray(...).array buffers (inputs and outputs) for the zero-copy path."""
        inputs = [np.ascontiguousarray(a) for a in inputs]
        if inputNum is None:
            inputNum = inputs[0].size * self.encDataPerPack
        n_out = self.getOutputSize(inputNum) // np.dtype(self.decPack_t).itemsize
        if outputs is None:
            outputs = [np.zeros(n_out, dtype=self.decPack_t) for _ in inputs]
        for a in inputs:
            if a.nbytes < self.getInputSize(inputNum):
                raise VitdecError("input buffer smaller than getInputSize(inputNum)")
        ins = (ctypes.c_void_p * len(inputs))(*[a.ctypes.data for a in inputs])
        outs = (ctypes.c_void_p * len(outputs))(*[o.ctypes.data for o in outputs])
        ms = ctypes.c_float(0.0)
        _check(lib().vd_run_stream(self._h, ins, outs, len(inputs), inputNum, ctypes.byref(ms)))
        return outputs, ms.value

    # ---- float channel values (SoftDecisionPacker(channel, scale) fused into the decode) ----
    def run_llr(self, llr_h, scale=40000.0, output_h=None):
        """Blocking decode of float channel values (viterbiDF.h:98-167 packer fused). Returns (out, ms)."""
        llr_h = np.ascontiguousarray(llr_h, dtype=np.float32)
        inputNum = llr_h.size
        if output_h is None:
            output_h = np.zeros(self.getOutputSize(inputNum) // np.dtype(self.decPack_t).itemsize,
                                dtype=self.decPack_t)
        ms = ctypes.c_float(0.0)
        _check(lib().vd_run_llr(self._h, llr_h.ctypes.data, output_h.ctypes.data, inputNum, scale, ctypes.byref(ms)))
        return output_h, ms.value

    def run_device_llr(self, llr_ptr, output_ptr, inputNum, scale=40000.0, stream=0):
        """Async fused decode of inputNum device floats (16-byte aligned)."""
        _check(lib().vd_run_device_llr(self._h, ctypes.c_void_p(llr_ptr), ctypes.c_void_p(output_ptr), inputNum,
                                       scale, ctypes.c_void_p(stream)))

    def run_device_llr_batch(self, llr_ptr, llr_stride, output_ptr, output_stride, inputNum, nbatch, scale=40000.0,
                             stream=0):
        """nbatch fused decodes of inputNum device floats each in one launch (vd_run_device_llr_batch)."""
        _check(lib().vd_run_device_llr_batch(self._h, ctypes.c_void_p(llr_ptr), llr_stride, ctypes.c_void_p(output_ptr),
                                             output_stride, inputNum, scale, nbatch, ctypes.c_void_p(stream)))


class PinnedArray:
    """A numpy view of page-locked host memory from vd_host_alloc (freed with the object)."""

    def __init__(self, shape, dtype):
        n = int(np.prod(shape)) * np.dtype(dtype).itemsize
        self._p = lib().vd_host_alloc(n)
        if not self._p:
            raise VitdecError("vd_host_alloc failed")
        buf = (ctypes.c_char * n).from_address(self._p)
        self.array = np.frombuffer(buf, dtype=dtype).reshape(shape)

    def __del__(self):
        if getattr(self, "_p", None):
            lib().vd_host_free(self._p)
            self._p = None


def pack_device(options, llr_ptr, inputNum, packed_ptr, scale=40000.0, stream=0):
    """The reference's SoftDecisionPacker on device floats -> vd_input_size(options, inputNum) bytes."""
    _check(lib().vd_pack_device(options, ctypes.c_void_p(llr_ptr), inputNum, scale, ctypes.c_void_p(packed_ptr),
                                ctypes.c_void_p(stream)))


def simulate_host(options, n_bits, snr, bit_seed, noise_seed):
    """Reference harness pipeline on the host (std::mt19937 + std::normal_distribution<float>)."""
    bits = np.zeros(n_bits, dtype=np.uint8)
    nbytes = lib().vd_input_size(options, 2 * n_bits)
    packed = np.zeros(nbytes // 4, dtype=np.float32 if (options & CHANNEL_MASK) == FP32 else np.int32)
    _check(lib().vd_simulate_host(options, n_bits, snr, bit_seed, noise_seed, bits.ctypes.data, packed.ctypes.data))
    return bits, packed


def channel_device(n_bits, snr, bit_seed, noise_seed, bits_ptr, values_ptr, stream=0):
    """The reference harness's RandBitGen | ConvolutionalEncoder | AddNoise on the GPU, bit-exact with
    simulate_host for the same seeds: n_bits bytes of message bits, 2 n_bits float channel values."""
    _check(lib().vd_channel_device(n_bits, snr, bit_seed, noise_seed, ctypes.c_void_p(bits_ptr),
                                   ctypes.c_void_p(values_ptr), ctypes.c_void_p(stream)))


def simulate_device(options, n_bits, snr, bit_seed, noise_seed, bits_ptr, packed_ptr, stream=0):
    """channel_device + SoftDecisionPacker(type, 40000): the packed input simulate_host makes, on the GPU."""
    _check(lib().vd_simulate_device(options, n_bits, snr, bit_seed, noise_seed,
                                    ctypes.c_void_p(bits_ptr) if bits_ptr else None, ctypes.c_void_p(packed_ptr),
                                    ctypes.c_void_p(stream)))


def split_redecodes(device=0):
    """split chunks re-decoded whole on a device so far (a speculative piece start did not converge)"""
    v = ctypes.c_uint64(0)
    _check(lib().vd_split_redecodes(device, ctypes.byref(v)))
    return v.value


def split_cap_exits(device=0):
    """split-launch waves that stopped re-decoding at the pass cap with a part still differing (always 0: the
    passes provably end within P; run / run_llr / run_stream raise if it is ever not)"""
    v = ctypes.c_uint64(0)
    _check(lib().vd_split_cap_exits(device, ctypes.byref(v)))
    return v.value


def mt_state_after(seed, n):
    """std::mt19937(seed)'s state array after n outputs (host GF(2) jump-ahead used by channel_device)."""
    st = np.zeros(624, dtype=np.uint32)
    _check(lib().vd_mt_state_after(seed, n, st.ctypes.data))
    return st


def count_errors(options, bits, decoded):
    return int(lib().vd_count_errors(options, bits.ctypes.data, bits.size, decoded.ctypes.data, decoded.nbytes))


def run_batches(options, inputs, inputNum, devices):
    """Independent batches sharded over `devices` (vd_run_batches). Returns (outputs, wall ms)."""
    n = len(inputs)
    dt = np.uint16 if (options & DECODE_MASK) == O_B16 else np.uint32
    outs = [np.zeros(lib().vd_output_size(options, inputNum) // np.dtype(dt).itemsize, dtype=dt) for _ in range(n)]
    ins = (ctypes.c_void_p * n)(*[x.ctypes.data for x in inputs])
    ous = (ctypes.c_void_p * n)(*[x.ctypes.data for x in outs])
    devs = (ctypes.c_int * len(devices))(*devices)
    ms = ctypes.c_float(0.0)
    _check(lib().vd_run_batches(options, ins, ous, inputNum, n, devs, len(devices), ctypes.byref(ms)))
    return outs, ms.value
