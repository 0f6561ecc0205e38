"""Experiment patch: K5's wave 0 raises its issue priority while it plans the block's rounds (the
block's first barrier waits on it).  usage: python3 plan_prio.py <csrc dir>"""
import os
import sys
p = os.path.join(sys.argv[1], "pf_kernels.hip")
s = open(p).read()
k0 = s.index("void fas_post_kernel(")
k1 = s.index("// ---------------------------------------------------------------- K2: merge")
k = s[k0:k1]
a = "        if (tid < 64) {  // read after the barrier below\n            wave_prefix(gpre, rng, H.n_tok, lane);"
assert k.count(a) == 1
k = k.replace(a, "        if (tid < 64) {  // read after the barrier below\n            __builtin_amdgcn_s_setprio(2);\n            wave_prefix(gpre, rng, H.n_tok, lane);", 1)
b = "                if (lane == 0) misc[3] = (uint32_t)nr;\n            }\n        }"
assert k.count(b) == 1
k = k.replace(b, "                if (lane == 0) misc[3] = (uint32_t)nr;\n            }\n            __builtin_amdgcn_s_setprio(0);\n        }", 1)
open(p, "w").write(s[:k0] + k + s[k1:])
