"""Experiment patch: merge_lists (pf_kernels.hip) prints its survivor counts (the first 40 calls).
usage: python3 mergedbg.py <csrc dir>"""
import os
import sys
p = os.path.join(sys.argv[1], "pf_kernels.hip")
s = open(p).read()
a = "    if (ns <= 64u) return wave_sort64(lane < (int)ns ? buf[lane] : ~0ull, lane);"
assert a in s
s = s.replace(a, """    {
        unsigned c = 0;
        if (lane == 0) c = atomicAdd(&g_mdbg, 1u);
        c = (unsigned)__builtin_amdgcn_readfirstlane((int)c);
        if (lane == 0 && c < 40u) printf("MERGEDBG nl %d k %d ns %u t0 %llx blk %d\\n", nl, k, ns, (unsigned long long)t0, (int)blockIdx.x);
    }
""" + a, 1)
s = s.replace("// the low n bits\n", "__device__ unsigned g_mdbg;\n// the low n bits\n", 1)
open(p, "w").write(s)
