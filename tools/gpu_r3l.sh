set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r3l && export TMPDIR=/tmp
PF_DEBUG=host_prof=1 timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'tools'); sys.path.insert(0,'recommendation-system-pokec_amd')
import time, synth, pokec_fas as pf
c=synth.Corpus(n_users=1632803, seed=1, threads=16)
d=c.desc_ptr()
import torch; torch.cuda.init(); torch.zeros(1).cuda()
t=time.time(); e=pf.FasEngine(d,0); print('pf_open (HIP initialised)', time.time()-t, flush=True); e.close()
" > gpurun_out/r3l/open_stages.txt 2>&1 || exit 6
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r3l/prof_cfg3 -o run -- python3 bench.py --workload cfg3 --steps 30 --warmup 3 --no-cpu-baseline --no-pmc > gpurun_out/r3l/cfg3_prof.json 2> gpurun_out/r3l/cfg3_prof.err || exit 4
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread -k "not full_size" > gpurun_out/r3l/gputest.log 2>&1 || exit 1
