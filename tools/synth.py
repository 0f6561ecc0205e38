"""ctypes wrapper of tools/libpokec_synth.so (seeded synthetic Pokec corpus).

Bench/test infrastructure.  `Corpus.desc_ptr()` is a pointer to a filled
`pf_corpus_desc` (include/pokec_fas.h) that can be handed to pf_open or to
the oracle without copying.
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libpokec_synth.so")


class PsParams(ctypes.Structure):
    _fields_ = [("n_users", ctypes.c_int32), ("n_cols", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("mean_degree", ctypes.c_double), ("vocab", ctypes.c_int32), ("n_club_ids", ctypes.c_int32),
                ("edge_cases", ctypes.c_int32), ("threads", ctypes.c_int32)]


def build():
    src = os.path.join(HERE, "pokec_synth.cpp")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["make", "-s", "-C", HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB)
        L.ps_generate.argtypes = [ctypes.POINTER(PsParams), ctypes.POINTER(ctypes.c_void_p)]
        L.ps_generate.restype = ctypes.c_int
        L.ps_desc.argtypes = [ctypes.c_void_p]
        L.ps_desc.restype = ctypes.c_void_p
        L.ps_median_age.argtypes = [ctypes.c_void_p]
        L.ps_median_age.restype = ctypes.c_int32
        L.ps_fill_ages.argtypes = [ctypes.c_void_p]
        L.ps_total_tokens.argtypes = [ctypes.c_void_p]
        L.ps_total_tokens.restype = ctypes.c_int64
        L.ps_write_reference_files.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.ps_write_reference_files.restype = ctypes.c_int
        L.ps_free.argtypes = [ctypes.c_void_p]
        _lib = L
    return _lib


class Corpus:
    """A generated corpus.  Ages are raw (0 = missing) until `fill_ages()`."""

    def __init__(self, n_users, seed=1, n_cols=48, edge_cases=0, mean_degree=18.75, vocab=2000,
                 n_club_ids=20000, threads=0):
        p = PsParams(n_users, n_cols, seed, mean_degree, vocab, n_club_ids, edge_cases, threads)
        h = ctypes.c_void_p()
        rc = lib().ps_generate(ctypes.byref(p), ctypes.byref(h))
        if rc != 0:
            raise RuntimeError(f"ps_generate failed ({rc})")
        self.h = h
        self.n_users = n_users
        self.filled = False

    def write_reference_files(self, root, normalizers=1, median=1):
        if self.filled:
            raise RuntimeError("write files before fill_ages()")
        rc = lib().ps_write_reference_files(self.h, root.encode(), int(normalizers), int(median))
        if rc != 0:
            raise RuntimeError("ps_write_reference_files failed")

    def fill_ages(self):
        if not self.filled:
            lib().ps_fill_ages(self.h)
            self.filled = True

    def desc_ptr(self):
        self.fill_ages()
        return lib().ps_desc(self.h)

    @property
    def median_age(self):
        return lib().ps_median_age(self.h)

    @property
    def total_tokens(self):
        return lib().ps_total_tokens(self.h)

    def close(self):
        if self.h:
            lib().ps_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
