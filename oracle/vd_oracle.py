"""ctypes front-end for the oracle library (TEST INFRASTRUCTURE ONLY).

The oracle is the CPU restatement of the reference decode path (see vd_oracle.c header for the
reference file:line map).  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
may import this module; the product never does.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libvd_oracle.so")
_lib = None

# option bits (reference src/viterbi/viterbi.h:7-20)
HARD, SOFT4, SOFT8, SOFT16, FP32 = 0x0, 0x1, 0x2, 0x3, 0x4
M_B32, M_B16, M_FP16 = 0x00, 0x10, 0x20
O_B32, O_B16 = 0x000, 0x100
REG, DPX = 0x0000, 0x1000


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        sz = ctypes.c_size_t
        L.vo_options_valid.argtypes = [ctypes.c_int]
        L.vo_input_size.argtypes = [ctypes.c_int, sz]
        L.vo_input_size.restype = sz
        L.vo_message_len.argtypes = [ctypes.c_int, sz]
        L.vo_message_len.restype = sz
        L.vo_output_size.argtypes = [ctypes.c_int, sz]
        L.vo_output_size.restype = sz
        L.vo_decode.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, sz, ctypes.c_int,
                                ctypes.c_int, ctypes.c_int]
        L.vo_simulate.argtypes = [ctypes.c_int, sz, ctypes.c_float, ctypes.c_uint32, ctypes.c_uint32,
                                  ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.vo_ben.argtypes = [ctypes.c_int, ctypes.c_void_p, sz, ctypes.c_void_p, sz]
        L.vo_pack.argtypes = [ctypes.c_int, ctypes.c_void_p, sz, ctypes.c_float, ctypes.c_void_p]
        L.vo_ben.restype = ctypes.c_longlong
        L.vo_gen_bits.argtypes = [ctypes.c_uint32, sz, ctypes.c_void_p]
        L.vo_gen_normals.argtypes = [ctypes.c_uint32, ctypes.c_float, sz, ctypes.c_void_p]
        L.vo_mt_raw.argtypes = [ctypes.c_uint32, sz, sz, ctypes.c_void_p]
        L.vo_logf_restated.argtypes = [ctypes.c_float]
        L.vo_logf_restated.restype = ctypes.c_float
        L.vo_logf_mismatch.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32]
        L.vo_logf_mismatch.restype = ctypes.c_longlong
        L.vo_channel.argtypes = [sz, ctypes.c_float, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                 ctypes.c_void_p, ctypes.c_void_p]
        L.vo_std_bits.argtypes = [ctypes.c_uint32, sz, ctypes.c_void_p]
        L.vo_std_normals.argtypes = [ctypes.c_uint32, ctypes.c_float, sz, ctypes.c_void_p]
        _lib = L
    return _lib


def options_valid(opt):
    return bool(lib().vo_options_valid(opt))


def input_size(opt, n):
    return lib().vo_input_size(opt, n)


def message_len(opt, n):
    return lib().vo_message_len(opt, n)


def output_size(opt, n):
    return lib().vo_output_size(opt, n)


def in_dtype(opt):
    return np.float32 if (opt & 0xF) == FP32 else np.int32


def out_dtype(opt):
    return np.uint16 if (opt & 0xF00) == O_B16 else np.uint32


def simulate(opt, n_bits, snr, bit_seed, noise_seed, noiseless=False):
    """Reference harness pipeline; returns (bits uint8[N], packed encPack_t array)."""
    bits = np.zeros(n_bits, dtype=np.uint8)
    nbytes = input_size(opt, 2 * n_bits)
    packed = np.zeros(nbytes // 4, dtype=in_dtype(opt))
    rc = lib().vo_simulate(opt, n_bits, snr, bit_seed, noise_seed, int(noiseless),
                           bits.ctypes.data, packed.ctypes.data)
    assert rc == 0
    return bits, packed


def _c_buffer(a, what):
    """a C-contiguous numpy array (the C side reads it through one pointer)"""
    if not isinstance(a, np.ndarray):
        raise ValueError(f"{what}: a numpy array is required, got {type(a).__name__}")
    if not a.flags.c_contiguous:
        raise ValueError(f"{what}: the array must be C-contiguous")
    return a


def decode(opt, packed, input_num=None, nchunks=6400, b16_policy=0, nthreads=None):
    """Decode like ViterbiCUDA<opt>::run; returns (decPack_t array, range_ok).

    Raises ValueError when `packed` holds fewer than input_size(opt, input_num) bytes: the C decoder reads
    that many, and a short buffer would be read past its end (round 4: a parity slice sized in packed words
    instead of bytes crashed the bench's parity block in decode_chunk)."""
    _c_buffer(packed, "decode")
    if input_num is None:
        per = {HARD: 32, SOFT4: 8, SOFT8: 4, SOFT16: 2, FP32: 1}[opt & 0xF]
        input_num = packed.size * per
    need = input_size(opt, input_num)
    if packed.nbytes < need:
        raise ValueError(f"decode: the input holds {packed.nbytes} bytes, option 0x{opt:x} with inputNum {input_num} "
                         f"reads {need}")
    out = np.zeros(output_size(opt, input_num) // np.dtype(out_dtype(opt)).itemsize, dtype=out_dtype(opt))
    if nthreads is None:
        nthreads = min(8, os.cpu_count() or 1)
    rc = lib().vo_decode(opt, packed.ctypes.data, out.ctypes.data, input_num, nchunks, b16_policy, nthreads)
    assert rc >= 0, rc
    return out, rc == 0


def pack(opt, values, scale=40000.0, input_num=None):
    """SoftDecisionPacker(channel, scale) on float32 channel values (viterbiDF.h:98-167).

    input_num: the channel values to pack (default: all of `values`); ValueError when `values` holds fewer."""
    if not isinstance(values, np.ndarray):
        raise ValueError(f"pack: a numpy array is required, got {type(values).__name__}")
    if input_num is not None:
        if values.size < input_num:
            raise ValueError(f"pack: {values.size} channel values given, inputNum {input_num}")
        values = values.reshape(-1)[:input_num]
    v = np.ascontiguousarray(values, dtype=np.float32)
    nbytes = input_size(opt, v.size)
    out = np.zeros((nbytes + 3) // 4, dtype=in_dtype(opt))
    lib().vo_pack(opt, v.ctypes.data, v.size, scale, out.ctypes.data)
    return out


def ben(opt, bits, dec):
    return int(lib().vo_ben(opt, bits.ctypes.data, bits.size, dec.ctypes.data, dec.nbytes))


def gen_bits(seed, n, use_std=False):
    out = np.zeros(n, dtype=np.uint8)
    (lib().vo_std_bits if use_std else lib().vo_gen_bits)(seed, n, out.ctypes.data)
    return out


def gen_normals(seed, stddev, n, use_std=False):
    out = np.zeros(n, dtype=np.float32)
    if use_std:
        lib().vo_std_normals(seed, stddev, n, out.ctypes.data)
    else:
        lib().vo_gen_normals(seed, stddev, n, out.ctypes.data)
    return out


def mt_raw(seed, n0, n):
    """raw std::mt19937(seed) outputs n0 .. n0+n-1"""
    out = np.zeros(n, dtype=np.uint32)
    lib().vo_mt_raw(seed, n0, n, out.ctypes.data)
    return out


def logf_mismatch(lo=0x00800000, hi=0x3F800000, stride=1):
    """count of floats (bit patterns lo..hi step stride) where the restated glibc logf != host logf"""
    return int(lib().vo_logf_mismatch(lo, hi, stride))


def channel(n_bits, snr, bit_seed, noise_seed, noiseless=False):
    """RandBitGen | ConvolutionalEncoder | AddNoise: (bits uint8[N], values float32[2N])"""
    bits = np.zeros(n_bits, dtype=np.uint8)
    vals = np.zeros(2 * n_bits, dtype=np.float32)
    lib().vo_channel(n_bits, snr, bit_seed, noise_seed, 1 if noiseless else 0, bits.ctypes.data, vals.ctypes.data)
    return bits, vals
