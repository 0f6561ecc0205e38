set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3k && export TMPDIR=/tmp
PF_DEBUG=host_prof=1 timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'tools'); sys.path.insert(0,'recommendation-system-pokec_amd')
import time, synth, pokec_fas as pf
c=synth.Corpus(n_users=1632803, seed=1, threads=16)
d=c.desc_ptr()
t=time.time(); e=pf.FasEngine(d,0); print('pf_open', time.time()-t, flush=True); e.close()
t=time.time(); e=pf.FasEngine(d,0); print('pf_open (second)', time.time()-t, flush=True); e.close()
" > gpurun_out/r3k/open_stages.txt 2>&1 || exit 6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3k/gputest.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --workload cfg3 --steps 60 --warmup 5 --no-cpu-baseline --no-pmc > gpurun_out/r3k/cfg3.json 2> gpurun_out/r3k/cfg3.err || exit 2
timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 1 --no-cpu-baseline --no-pmc > gpurun_out/r3k/cfg5_c1.json 2> gpurun_out/r3k/cfg5_c1.err || exit 3
timeout -k 10 600 python3 bench.py --workload cfg5 --steps 5 --warmup 2 --contexts 3 --no-cpu-baseline --no-pmc > gpurun_out/r3k/cfg5_c3.json 2> gpurun_out/r3k/cfg5_c3.err || exit 4
