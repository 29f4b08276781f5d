"""ctypes binding of the CPU oracle (oracle/lz4ada_oracle.c).

Test infrastructure: the checker, never the thing measured or shipped.
"""
import ctypes
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "oracle", "_build", "liblz4ada_oracle.so")

OK, CHECKSUM_ERROR, DATA_CORRUPTION, NOT_SUPPORTED = 0, 1, 2, 3
TOO_FEW_HEADER_BYTES, TOO_LITTLE_MEMORY = 4, 5
SZ_64_KIB, SZ_256_KIB, SZ_1_MIB, SZ_4_MIB, SZ_8_MIB, USE_FIRST, SINGLE_FRAME = range(7)
FOR_ALL = SZ_8_MIB
EOF_YES, EOF_NO, EOF_MAYBE = 0, 1, 2

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB)
        i64, p = ctypes.c_int64, ctypes.c_void_p
        pi64 = ctypes.POINTER(ctypes.c_int64)
        L.oracle_init.argtypes = [ctypes.c_int, pi64, ctypes.POINTER(p)]
        L.oracle_init_with_header.argtypes = [ctypes.c_char_p, i64, ctypes.c_int, pi64, pi64,
                                              ctypes.POINTER(p), ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_init_for_block.argtypes = [i64, ctypes.c_int, pi64, ctypes.POINTER(p)]
        L.oracle_update.argtypes = [p, ctypes.c_void_p, i64, pi64, ctypes.c_void_p, i64, pi64, pi64]
        L.oracle_is_end_of_frame.argtypes = [p]
        L.oracle_last_error.argtypes = [p]
        L.oracle_last_error.restype = ctypes.c_char_p
        L.oracle_error_name.argtypes = [ctypes.c_int]
        L.oracle_error_name.restype = ctypes.c_char_p
        L.oracle_free.argtypes = [p]
        L.oracle_xxh32_hash.argtypes = [ctypes.c_char_p, i64]
        L.oracle_xxh32_hash.restype = ctypes.c_uint32
        L.oracle_xxh32_init.argtypes = [p, ctypes.c_uint32]
        L.oracle_xxh32_reset.argtypes = [p, ctypes.c_uint32]
        L.oracle_xxh32_update.argtypes = [p, ctypes.c_char_p, i64]
        L.oracle_xxh32_final.argtypes = [p]
        L.oracle_xxh32_final.restype = ctypes.c_uint32
        L.oracle_decode_stream.argtypes = [ctypes.c_char_p, i64, i64, ctypes.c_int, ctypes.c_void_p,
                                           i64, pi64, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p,
                                           ctypes.c_size_t]
        L.oracle_error_harness.argtypes = [ctypes.c_char_p, i64, ctypes.c_char_p, ctypes.c_size_t]
        L.oracle_unlz4ada.argtypes = [ctypes.c_char_p, i64, ctypes.c_void_p, i64, pi64,
                                      ctypes.c_char_p, ctypes.c_size_t]
        _lib = L
    return _lib


def error_name(status: int) -> str:
    return lib().oracle_error_name(status).decode()


def exception_information(status: int, msg: str) -> str:
    """The reference's Exception_Information line (lz4test.adb:312-313)."""
    return f"raised {error_name(status)} : {msg}"


def decode_stream(data: bytes, chunk: int = 4096, reservation: int = FOR_ALL, out_cap=None):
    """lz4test.adb:32-83 feed loop; returns (status, output, eof, message)."""
    cap = out_cap if out_cap is not None else max(64 << 20, 4 * len(data) + (16 << 20))
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_int64()
    eof = ctypes.c_int()
    err = ctypes.create_string_buffer(512)
    st = lib().oracle_decode_stream(data, len(data), chunk, reservation, out, cap,
                                    ctypes.byref(n), ctypes.byref(eof), err, 512)
    return st, out.raw[:n.value], eof.value, err.value.decode()


def error_harness(data: bytes):
    err = ctypes.create_string_buffer(512)
    st = lib().oracle_error_harness(data, len(data), err, 512)
    return st, err.value.decode()


def unlz4ada(data: bytes, out_cap=None):
    cap = out_cap if out_cap is not None else max(64 << 20, 4 * len(data))
    out = ctypes.create_string_buffer(cap)
    n = ctypes.c_int64()
    err = ctypes.create_string_buffer(512)
    st = lib().oracle_unlz4ada(data, len(data), out, cap, ctypes.byref(n), err, 512)
    return st, out.raw[:n.value], err.value.decode()


def xxh32(data: bytes) -> int:
    return lib().oracle_xxh32_hash(data, len(data))


class XXH32:
    """LZ4Ada.XXHash32 (lz4ada.ads:311-344) over the oracle."""

    def __init__(self, seed: int = 0):
        self._st = ctypes.create_string_buffer(48)
        lib().oracle_xxh32_init(self._st, seed)

    def reset(self, seed: int = 0):
        lib().oracle_xxh32_reset(self._st, seed)

    def update(self, data: bytes):
        lib().oracle_xxh32_update(self._st, data, len(data))

    def final(self) -> int:
        return lib().oracle_xxh32_final(self._st)


class Decompressor:
    """Streaming context over the oracle (mirrors lz4ada.ads:189-303)."""

    def __init__(self, ptr, min_buffer_size):
        self._p = ctypes.c_void_p(ptr)
        self.min_buffer_size = min_buffer_size

    def __del__(self):
        if getattr(self, "_p", None) and self._p.value:
            lib().oracle_free(self._p)

    @classmethod
    def init(cls, reservation=FOR_ALL):
        mbs = ctypes.c_int64()
        p = ctypes.c_void_p()
        st = lib().oracle_init(reservation, ctypes.byref(mbs), ctypes.byref(p))
        assert st == OK
        return cls(p.value, mbs.value)

    @classmethod
    def init_with_header(cls, data: bytes, reservation=SINGLE_FRAME):
        mbs = ctypes.c_int64()
        cons = ctypes.c_int64()
        p = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        st = lib().oracle_init_with_header(data, len(data), reservation, ctypes.byref(cons),
                                           ctypes.byref(mbs), ctypes.byref(p), err, 512)
        if st:
            return st, err.value.decode(), None, None
        return OK, "", cls(p.value, mbs.value), cons.value

    @classmethod
    def init_for_block(cls, compressed_length, reservation=FOR_ALL):
        mbs = ctypes.c_int64()
        p = ctypes.c_void_p()
        st = lib().oracle_init_for_block(compressed_length, reservation, ctypes.byref(mbs),
                                         ctypes.byref(p))
        assert st == OK
        return cls(p.value, mbs.value)

    def update(self, data: bytes, buf):
        """Returns (status, consumed, first, last); buf is a ctypes buffer."""
        cons, f, l = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        src = ctypes.create_string_buffer(data, len(data)) if data else None
        st = lib().oracle_update(self._p, src, len(data), ctypes.byref(cons), buf,
                                 len(buf), ctypes.byref(f), ctypes.byref(l))
        return st, cons.value, f.value, l.value

    def last_error(self) -> str:
        return lib().oracle_last_error(self._p).decode()

    def is_end_of_frame(self) -> int:
        return lib().oracle_is_end_of_frame(self._p)
