"""Experiment patch: K5 builds the next round's list map inside the walk (wave 0, after the round's
entry loads are issued and before their first use), so the map's LDS work overlaps the loads'
latency instead of running between the walk barrier and the slots barrier, where waves 1-3 wait
for it.  usage: python3 mapearly.py <csrc dir>"""
import os
import sys
p = os.path.join(sys.argv[1], "pf_kernels.hip")
s = open(p).read()
a = """                        kn[u] = ps.pnorm[K5CHK(xs[u], ps.n_tok_entries, 5)];
                    }
"""
assert s.count(a) == 1
s = s.replace(a, a + """                    if (tid < 64 && rnd + 1 < nrounds) {  // [mapearly] the next round's list map, loads in flight
                        const uint2 r1 = rtab[rnd + 1];
                        const int nb = mbuf ^ 1;
                        build_map(mapb + nb * kMapWords, mapc + nb * kMapWords, mapn + nb * kRoundToks, gpre, rng,
                                  (int)(r1.x & 0xFFFFu), (int)(r1.x >> 16), lane);
                    }
""", 1)
b = """                if (tid < 64 && rnd + 1 < nrounds) {  // the next round's list map (published by the slots barrier)
                    const uint2 r1 = rtab[rnd + 1];
                    const int nb = mbuf ^ 1;
                    build_map(mapb + nb * kMapWords, mapc + nb * kMapWords, mapn + nb * kRoundToks, gpre, rng,
                              (int)(r1.x & 0xFFFFu), (int)(r1.x >> 16), lane);
                }
"""
assert s.count(b) == 1
s = s.replace(b, "", 1)
open(p, "w").write(s)
