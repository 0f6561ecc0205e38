"""Experiment patch: K5 waves set their issue priority by dispatch order (bx / (nbx / 4)), so the
workgroups dispatched last on a CU are not starved by age-ordered arbitration.
PRIO=up (later dispatched = higher), PRIO=flat2 (all 2).  usage: python3 prio.py <csrc dir>"""
import os
import sys
p = os.path.join(sys.argv[1], "pf_kernels.hip")
s = open(p).read()
k0 = s.index("void fas_post_kernel(")
k1 = s.index("// ---------------------------------------------------------------- K2: merge")
k = s[k0:k1]
a = "    const uint8_t* img = pool + img_off[qy];\n    const QPostHead H = *reinterpret_cast<const QPostHead*>(img + sizeof(QConst));"
assert k.count(a) == 1
mode = os.environ.get("PRIO", "up")
if mode == "up":
    ins = """    {
        const int slot4 = min(3, bx / max(1, nbx >> 2));
        if (slot4 == 1) __builtin_amdgcn_s_setprio(1);
        else if (slot4 == 2) __builtin_amdgcn_s_setprio(2);
        else if (slot4 == 3) __builtin_amdgcn_s_setprio(3);
    }
"""
else:
    ins = "    __builtin_amdgcn_s_setprio(2);\n"
k = k.replace(a, ins + a, 1)
open(p, "w").write(s[:k0] + k + s[k1:])
