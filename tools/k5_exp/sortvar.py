"""Experiment patches of the wave sort (pf_device.h): SORTVAR=shfl -> every lane exchange by
__shfl_xor (ds_bpermute); SORTVAR=noinl -> wave_sort64 out of line.  usage: python3 sortvar.py <csrc dir>"""
import os
import sys
p = os.path.join(sys.argv[1], "pf_device.h")
s = open(p).read()
v = os.environ.get("SORTVAR", "")
if v == "shfl":
    assert "    switch (m) {" in s
    s = s.replace("    switch (m) {", "    switch (m + 1000) {", 1)
elif v == "noinl":
    a = "__device__ __forceinline__ uint64_t wave_sort64(uint64_t x, int lane) {"
    assert a in s
    s = s.replace(a, "static __device__ __attribute__((noinline)) uint64_t wave_sort64(uint64_t x, int lane) {", 1)
else:
    sys.exit("SORTVAR=shfl|noinl")
open(p, "w").write(s)
