#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REAL reference.

TEST INFRASTRUCTURE ONLY — runs in the build container, where /root/reference
exists.  Steps:
  1. tools/libpokec_synth.so writes seeded synthetic corpora in the reference's
     own on-disk formats (users_encoded.csv, adjacency.csv, ...);
  2. oracle/_ref/ref_fixture (the reference compiled from its own sources by
     oracle/Makefile, linked with a harness) loads each corpus exactly like
     api_cli does and dumps parsed profiles, IDF, FAS pairs, recommender
     outputs, all-candidates top-50 and hold-out driver results;
  3. oracle/_ref/api_cli (the reference's own CLI) answers a scripted stdin
     transcript (PING / USER / unknown / empty / EXIT);
  4. everything is gzip'd into tests/golden/<corpus>/.

The corpora themselves are NOT committed: tests regenerate them bit-identically
from the same generator + parameters (recorded in tests/golden/manifest.json).

usage: python oracle/gen_golden.py [--norms-only]   (needs `make -C oracle ref` and `make -C tools`)
"""
import gzip
import json
import os
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")

# name -> generator params + writer options + harness options
CORPORA = {
    "A": dict(n_users=2500, seed=11, edge_cases=1, normalizers=1, median=1,
              npairs=60000, pair_seed=7, holdout=12, rectest=6, digest_holdout=60, digest_rectest=120),
    "B": dict(n_users=1200, seed=23, edge_cases=1, normalizers=0, median=0,
              npairs=20000, pair_seed=9, holdout=0, rectest=0, digest_holdout=0, digest_rectest=0),
}
# config 1 plumbing (BASELINE.json configs[0]): api_cli with load_users=10000
API_CORPUS = dict(n_users=10000, seed=31, edge_cases=0, normalizers=1, median=1)


def run_harness(work, out, c):
    exe = os.path.join(HERE, "_ref", "ref_fixture")
    with open(os.path.join(out, "harness_stdout.txt"), "w") as so:
        subprocess.run([exe, work, out, str(c["npairs"]), str(c["pair_seed"]),
                        str(c["holdout"]), str(c["rectest"]), str(c["digest_holdout"]), str(c["digest_rectest"])],
                       check=True, stdout=so)
    os.remove(os.path.join(out, "harness_stdout.txt"))


def transcript_for(work, uids, load_users="10000"):
    exe = os.path.join(HERE, "_ref", "api_cli")
    lines = ["PING", ""] + [f"USER {u}" for u in uids] + ["USER 999999999", "USER -3",
                                                         "FOO 1", "USER", "EXIT", "PING"]
    stdin = "\n".join(lines) + "\n"
    r = subprocess.run([exe, load_users], cwd=work, input=stdin.encode(), capture_output=True, check=True)
    return lines, r.stdout.decode()


# compute_column_normalizers goldens (A18): corpus -> (sample_size, comps_per_user)
NORM_RUNS = {"A": (3000, 5), "B": (1500, 3)}


def gen_norms():
    """ref_norms on corpora A and B: the CSV save_column_normalizers writes and the
    (mean, sd) float bits, as tests/golden/<corpus>/norms_computed_{csv,bits}.txt.gz."""
    exe = os.path.join(HERE, "_ref", "ref_norms")
    for name, (sample, comps) in NORM_RUNS.items():
        c = CORPORA[name]
        out = os.path.join(GOLDEN, name)
        with tempfile.TemporaryDirectory() as work, tempfile.TemporaryDirectory() as raw:
            corpus = synth.Corpus(n_users=c["n_users"], seed=c["seed"], edge_cases=c["edge_cases"])
            corpus.write_reference_files(work, normalizers=c["normalizers"], median=c["median"])
            corpus.close()
            csv, bits = os.path.join(raw, "norms_computed_csv.txt"), os.path.join(raw, "norms_computed_bits.txt")
            subprocess.run([exe, work, csv, bits, str(sample), str(comps)], check=True, stdout=subprocess.DEVNULL)
            for fn in (csv, bits):
                gz_copy(fn, os.path.join(out, os.path.basename(fn) + ".gz"))
        print("norms", name, "done", file=sys.stderr)


def gz_copy(src, dst):
    with open(src, "rb") as fi, open(dst, "wb") as raw, \
            gzip.GzipFile(fileobj=raw, mode="wb", compresslevel=9, mtime=0) as fo:
        shutil.copyfileobj(fi, fo)


def main():
    os.makedirs(GOLDEN, exist_ok=True)
    if "--norms-only" in sys.argv:
        gen_norms()
        return
    manifest = {"generator": "tools/pokec_synth.cpp", "corpora": {}, "api_cli": {}}
    for name, c in CORPORA.items():
        out = os.path.join(GOLDEN, name)
        os.makedirs(out, exist_ok=True)
        with tempfile.TemporaryDirectory() as work, tempfile.TemporaryDirectory() as raw:
            corpus = synth.Corpus(n_users=c["n_users"], seed=c["seed"], edge_cases=c["edge_cases"])
            corpus.write_reference_files(work, normalizers=c["normalizers"], median=c["median"])
            corpus.close()
            run_harness(work, raw, c)
            for fn in sorted(os.listdir(raw)):
                gz_copy(os.path.join(raw, fn), os.path.join(out, fn + ".gz"))
        manifest["corpora"][name] = c
        print("corpus", name, "done", file=sys.stderr)

    out = os.path.join(GOLDEN, "api")
    os.makedirs(out, exist_ok=True)
    with tempfile.TemporaryDirectory() as work:
        corpus = synth.Corpus(n_users=API_CORPUS["n_users"], seed=API_CORPUS["seed"],
                              edge_cases=API_CORPUS["edge_cases"])
        corpus.write_reference_files(work, normalizers=API_CORPUS["normalizers"], median=API_CORPUS["median"])
        corpus.close()
        uids = [1, 2, 17, 4242, 9999, 10000]
        lines, stdout = transcript_for(work, uids)
        with gzip.open(os.path.join(out, "transcript_stdin.txt.gz"), "wt", compresslevel=9) as f:
            f.write("\n".join(lines) + "\n")
        with gzip.open(os.path.join(out, "transcript_stdout.txt.gz"), "wt", compresslevel=9) as f:
            f.write(stdout)
    manifest["api_cli"] = dict(API_CORPUS, load_users="10000", uids=uids)
    gen_norms()
    manifest["norm_runs"] = {k: list(v) for k, v in NORM_RUNS.items()}
    with open(os.path.join(GOLDEN, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("golden fixtures written to", GOLDEN, file=sys.stderr)


if __name__ == "__main__":
    main()
