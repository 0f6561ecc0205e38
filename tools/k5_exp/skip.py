"""Phase-skip experiment patches of K5 (fas_post_kernel) for variant builds: each removes one
piece of work (the results are wrong; time only).  usage: SKIP=a,b python3 skip.py <csrc dir>"""
import os
import sys

d = sys.argv[1]
p = os.path.join(d, "pf_kernels.hip")
s = open(p).read()
a = s.index("void fas_post_kernel(")
b = s.index("// ---------------------------------------------------------------- K2: merge")
k = s[a:b]


def rep(old, new):
    global k
    assert old in k, old[:80]
    k = k.replace(old, new)


for what in os.environ.get("SKIP", "").split(","):
    if what == "terms":  # no cosine -> sigmoid (the FP64 divisions and exp of every item)
        rep("slot[r] = dot == 0.0 ? q.sig0_col[t] : text_term(q, t, dot, nrm);", "slot[r] = dot + nrm;")
    elif what == "items":  # no item compaction and terms at all
        rep("for (uint32_t r0 = wb; r0 < wb + wn; r0 += 64) {", "for (uint32_t r0 = wb; r0 < wb; r0 += 64) {")
    elif what == "fas":  # no FAS divisions
        rep("f = (S <= 0.0 && Fv <= 0.0) ? 0.0f : (float)((2.0 * S * Fv) / (S + Fv));", "f = (float)(S + Fv);")
        rep("const double S = sum[kk] / (double)uk;", "const double S = sum[kk];")
    elif what == "owner":  # no owner sums
        rep("for (uint64_t pr = pend[kk] & rtm; pr; pr &= pr - 1) {", "for (uint64_t pr = 0; pr; pr &= pr - 1) {")
    elif what == "place":  # no hit placing
        rep("                    if (kp[u] == ~0u) continue;\n                    const uint32_t p = kp[u] & 1023u",
            "                    if (kp[u] != 12345u) continue;\n                    const uint32_t p = kp[u] & 1023u")
    elif what == "merge":  # no fused cross-block merge
        rep("    post_tail(best, k, sc,", "    if (lane < k) parts[bx * k + lane] = best;\n    return;\n    post_tail(best, k, sc,")
    elif what == "sets":  # no club / friend lists
        rep("        walk_sets(ps, rng + H.n_tok, nsets,", "        walk_sets(ps, rng + H.n_tok, 0,")
    elif what == "text":  # no text rounds at all
        rep("        int nrounds = (int)misc[3];", "        int nrounds = 0;")
    elif what:
        sys.exit(f"unknown skip {what}")
s = s[:a] + k + s[b:]
open(p, "w").write(s)
