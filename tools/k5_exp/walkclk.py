"""Experiment patch (with K5T=1): K5's walk split into finer clocks — the list-map lookups (slot 14),
the entry loads up to their arrival (slot 16: an explicit vmcnt(0) wait after the issue) and the
mask atomics (slot 17); the rest of the walk stays in slot 4.  usage: python3 walkclk.py <csrc dir>"""
import os
import sys
p = os.path.join(sys.argv[1], "pf_kernels.hip")
s = open(p).read()
s = s.replace("__device__ unsigned long long g_k5t[16];", "__device__ unsigned long long g_k5t[20];", 1)
s = s.replace("    uint64_t tacc[14] = {0};", "    uint64_t tacc[20] = {0};", 1)
s = s.replace("        for (int i = 0; i < 14; ++i) atomicAdd(&g_k5t[i], (unsigned long long)tacc[i]);",
              "        for (int i = 0; i < 20; ++i) if (i != 15) atomicAdd(&g_k5t[i], (unsigned long long)tacc[i]);", 1)
a = "                    uint32_t ent[U];\n"
assert s.count(a) == 1
s = s.replace(a, "                    K5T(14);\n" + a, 1)
b = """                        kn[u] = ps.pnorm[K5CHK(xs[u], ps.n_tok_entries, 5)];
                    }
"""
assert s.count(b) == 1
s = s.replace(b, b + """                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    K5T(16);
""", 1)
c = """                            atomicOr(reinterpret_cast<unsigned long long*>(&mask[p]), 1ull << jr);
                        }
                    }
                }
"""
assert s.count(c) == 1
s = s.replace(c, c + "                K5T(17);\n", 1)
# the host report: 20 slots
s = s.replace("        unsigned long long t[16];\n        hipStreamSynchronize(s);\n        hipMemcpyFromSymbol(t, HIP_SYMBOL(g_k5t), sizeof(t));",
              "        unsigned long long t[20];\n        hipStreamSynchronize(s);\n        hipMemcpyFromSymbol(t, HIP_SYMBOL(g_k5t), sizeof(t));", 1)
i = s.index('static const char* nm[14] = {"ranges+hdr"')
j = s.index("const unsigned long long z[16] = {0};", i)
seg = s[i:j]
seg2 = seg.replace("static const char* nm[14]", "static const char* nm[20]")
seg2 = seg2.replace('"total"}', '"total", "walk-map", "cnt", "walk-load", "walk-atomics", "-", "-"}')
seg2 = seg2.replace("for (int i = 0; i < 14; ++i)", "for (int i = 0; i < 18; ++i) if (i != 15)")
s = s[:i] + seg2 + s[j:].replace("const unsigned long long z[16] = {0};", "const unsigned long long z[20] = {0};", 1)
open(p, "w").write(s)
