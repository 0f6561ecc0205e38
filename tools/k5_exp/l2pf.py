"""Experiment patch: L2 prefetch of K5's next-round walk entries.  Once the next round's list map is
published (the slots barrier), each lane issues one post-entry load and one norm-word load spread
over its wave's chunks of the next round (lane l: chunk l % U, offset 6 (l / U): every 128-B line
of the chunk's entries and norms is touched), held in two VGPRs and consumed (an empty asm) at the
next round's walk, so the walk's own loads hit L2.  PF_POS=place (default: issued at the place
phase, after the slots barrier) or terms (after the place barrier).  usage: python3 l2pf.py <csrc dir>"""
import os
import sys
p = os.path.join(sys.argv[1], "pf_kernels.hip")
s = open(p).read()
pos = os.environ.get("PF_POS", "place")
pf = """                if (rnd + 1 < nrounds) {  // [experiment l2pf] the next round's lines into L2
                    const uint2 r1n = rtab[rnd + 1];
                    const int ja1 = (int)(r1n.x & 0xFFFFu), jb1 = (int)(r1n.x >> 16);
                    const uint32_t F1 = gpre[jb1] - gpre[ja1];
                    const uint32_t fp = (uint32_t)(tid & ~63) + (uint32_t)kPostThreads * (uint32_t)(lane % U) + 6u * (uint32_t)(lane / U);
                    if (fp < F1 && fp < (uint32_t)kRoundCap) {
                        const int nb1 = mbuf ^ 1;
                        const uint32_t w1 = fp >> 6;
                        const uint32_t kk1 = (uint32_t)mapc[nb1 * kMapWords + w1] +
                                             (uint32_t)__popcll(mapb[nb1 * kMapWords + w1] & low_bits((fp & 63u) + 1u)) - 1u;
                        const uint32_t x1 = mapn[nb1 * kRoundToks + kk1].x + fp;
                        pf_a = ps.post[x1];
                        pf_b = reinterpret_cast<const uint32_t*>(ps.pnorm)[2 * (size_t)x1];
                    }
                }
"""
anchor = ("                // c. place every hit at its slot, the column's first hit with its norm\n" if pos == "place"
          else "                // d. terms, one (candidate, column) item per lane over the wave's slots\n")
assert s.count(anchor) == 1
s = s.replace(anchor, anchor + pf, 1)
# U is declared inside the walk block scope: make it visible (constexpr at the round's scope)
a = "                constexpr int U = kRoundCap / kPostThreads;\n"
assert s.count(a) == 1
s = s.replace(a, "", 1)
b = "        for (int rnd = 0; rnd < nrounds; ++rnd) {\n"
assert s.count(b) == 1
s = s.replace(b, "        constexpr int U = kRoundCap / kPostThreads;\n        uint32_t pf_a = 0u, pf_b = 0u;\n" + b, 1)
c = "                // a. walk: the round's entries flattened over the workgroup, all loads in flight\n"
assert s.count(c) == 1
s = s.replace(c, c + '                asm volatile("" :: "v"(pf_a), "v"(pf_b));\n', 1)
open(p, "w").write(s)
