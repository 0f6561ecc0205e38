set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3j && export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3j/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3j/cfg3.json 2> gpurun_out/r3j/cfg3.err || exit 2
PF_DEBUG=host_prof=1 timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'tools'); sys.path.insert(0,'recommendation-system-pokec_amd')
import time, synth, pokec_fas as pf
c=synth.Corpus(n_users=1632803, seed=1, threads=16)
d=c.desc_ptr()
t=time.time(); e=pf.FasEngine(d,0); print('pf_open', time.time()-t, flush=True); e.close()
" > gpurun_out/r3j/open_stages.txt 2>&1 || exit 6
bash tools/pmc_passes.sh r3j_k1p fas_pairs --workload cfg3 > gpurun_out/r3j/pmc.log 2>&1 || exit 3
make -C recommendation-system-pokec_amd clean > /dev/null && make -C recommendation-system-pokec_amd -j16 K5T=1 > gpurun_out/r3j/build_k5t.log 2>&1 || exit 4
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3j/cfg3_k5t.json 2> gpurun_out/r3j/cfg3_k5t.err || exit 5
