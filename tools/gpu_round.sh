# One parameterised GPU-box script for the round's runs (replaces the per-run tools/gpu_r3*.sh).
#   bash tools/gpu_round.sh TAG STEP [STEP ...]
# Steps (each under its own time limit, chained: the first failure ends the script):
#   tests        full GPU suite                         -> gpurun_out/TAG/gputest.log
#   tests:EXPR   GPU tests matching -k EXPR             -> gpurun_out/TAG/gputest_k.log
#   testse:E     full GPU suite under PF_DEBUG=E        -> gpurun_out/TAG/gputest_e.log
#   bench        default bench line (cfg 2, CPU baseline + PMC pass) -> bench.json
#   prof         rocprofv3 kernel trace + stats of a 20-step cfg-2 run -> prof_default/
#   cfgN         bench.py --workload cfgN               -> cfgN.json
#   quick        cfg 2, 100 steps, no CPU baseline / PMC -> quick.json
#   quick4       cfg 4, 3 steps, no CPU baseline / PMC   -> quick4.json
#   forcedist    cfg 2 through the N > 1 step at world 1 (RCCL communicator + all-gather) -> forcedist.json
#   quickv:V / quick4v:V  the same with the variant library vlib/V (tools/build_variant.sh)
#   cfg5c1       cfg 5 at one context with the host stage clocks (PF_DEBUG host_prof=1) -> cfg5c1.err
#   k5t          profiling build (tools/build_variant.sh k5t K5T=1 -> vlib/k5t) per-phase K5 clocks -> k5t.err
#   pmc:NAME:C1,C2..  one rocprofv3 --pmc pass over a 20-step cfg-2 run -> pmc_NAME/
#   ab:W:N:R:A/B  alternating A/B bench lines (replaces the per-run tools/r*.sh scripts of rounds 4-5):
#                 workload W (cfg2..cfg5), N timed steps, R pairs; A and B are each "-" (the default
#                 tree), a PF_DEBUG setting (e.g. k5_dyn=0), or lib=V (the variant library vlib/V);
#                 every line appended to ab_W.txt as "A|B <json>"
#   trace:N       rocprofv3 kernel trace (csv, no stats) of an N-step cfg-2 run -> trace/
set -o pipefail
TAG=$1
shift
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/$TAG && export TMPDIR=/tmp
O=gpurun_out/$TAG
Q="--no-cpu-baseline --no-pmc"
for S in "$@"; do
    echo "== $S $(date +%T)"
    case $S in
    tests)
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest.log 2>&1 || exit 1 ;;
    testse:*)
        # the full GPU suite under PF_DEBUG=SETTINGS (e.g. testse:k5_slice=1)
        E=${S#testse:}
        timeout -k 10 900 env PF_DEBUG=$E python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread > $O/gputest_e.log 2>&1 || exit 1 ;;
    tests:*)
        timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${S#tests:}" > $O/gputest_k.log 2>&1 || exit 1 ;;
    bench)
        timeout -k 10 600 python3 bench.py > $O/bench.json 2> $O/bench.err || exit 2 ;;
    prof)
        timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_default -o run -- python3 bench.py --steps 20 --warmup 5 $Q > $O/prof.json 2> $O/prof.err || exit 3 ;;
    cfg3h|cfg3h:*)
        # cfg 3 with the host stage clocks; cfg3h:K runs K timed steps (default 50)
        K=50; [[ $S == cfg3h:* ]] && K=${S#cfg3h:}
        timeout -k 10 600 env PF_DEBUG=host_prof=1 python3 bench.py --workload cfg3 --steps $K --warmup 5 $Q > $O/cfg3h_$K.json 2> $O/cfg3h_$K.err || exit 4 ;;
    prof3)
        # kernel trace of cfg 3 (the asynchronous pair-kernel pipeline at one context)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof_cfg3 -o run -- python3 bench.py --workload cfg3 --steps 30 --warmup 5 $Q > $O/prof3.json 2> $O/prof3.err || exit 3 ;;
    prof5)
        # kernel trace of cfg 5 at one context (host-side gaps between the device stages)
        timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/prof_cfg5 -o run -- python3 bench.py --workload cfg5 --contexts 1 --steps 5 --warmup 2 $Q > $O/prof5.json 2> $O/prof5.err || exit 3 ;;
    cfg[2345])
        timeout -k 10 900 python3 bench.py --workload $S > $O/$S.json 2> $O/$S.err || exit 4 ;;
    quick)
        timeout -k 10 300 python3 bench.py --steps 100 --warmup 10 $Q > $O/quick.json 2> $O/quick.err || exit 5 ;;
    quickv:*)
        V=${S#quickv:}
        timeout -k 10 300 env PF_LIB_PATH=$PWD/vlib/$V/libpokec_fas.so python3 bench.py --steps 100 --warmup 10 $Q > $O/quick_$V.json 2> $O/quick_$V.err || exit 5 ;;
    varchk:*)
        # varchk:V  tests/gpu_variant_check.py (oracle-checked batched and one-query calls) with vlib/V,
        # at the default launch and with 16-workgroup one-query launches (several claimed blocks each)
        V=${S#varchk:}
        timeout -k 10 300 env PF_LIB_PATH=$PWD/vlib/$V/libpokec_fas.so python3 tests/gpu_variant_check.py > $O/varchk_$V.log 2>&1 &&
        timeout -k 10 300 env PF_LIB_PATH=$PWD/vlib/$V/libpokec_fas.so PF_DEBUG=k5_wgs=16 python3 tests/gpu_variant_check.py >> $O/varchk_$V.log 2>&1 || exit 14
        echo "varchk $V ok" >> $O/varchk_$V.log ;;
    quick4v:*)
        V=${S#quick4v:}
        timeout -k 10 300 env PF_LIB_PATH=$PWD/vlib/$V/libpokec_fas.so python3 bench.py --workload cfg4 --steps 3 --warmup 1 $Q > $O/quick4_$V.json 2> $O/quick4_$V.err || exit 6 ;;
    quickd:*|quick4d:*)
        # the same quick lines from another tree (e.g. a git worktree of an older commit under exp/)
        D=${S#*:}; N=$(basename $D); W=""; [[ $S == quick4d:* ]] && W="--workload cfg4 --steps 3 --warmup 1" || W="--steps 100 --warmup 10"
        (cd $D && timeout -k 10 300 python3 bench.py $W $Q) > $O/${S%%:*}_$N.json 2> $O/${S%%:*}_$N.err || exit 6 ;;
    whole5)
        # cfg 5 over EVERY eligible user of the 1.63M corpus (both drivers), prefix-checked
        timeout -k 10 1000 python3 -u tools/eval_holdout.py --cfg5-corpus 1632803 --whole --check-prefix 64 \
            --out $O/whole5.json > $O/whole5.log 2>&1 || exit 10 ;;
    quicke:*)
        # cfg 2 quick line under a PF_DEBUG setting
        E=${S#quicke:}
        timeout -k 10 300 env PF_DEBUG=$E python3 bench.py --steps 100 --warmup 10 $Q > $O/quicke_${E//[=,]/_}.json 2> $O/quicke.err || exit 5 ;;
    quick4e:*)
        # cfg 4 quick line under a PF_DEBUG setting, e.g. quick4e:k5_query_major=1
        E=${S#quick4e:}
        timeout -k 10 300 env PF_DEBUG=$E python3 bench.py --workload cfg4 --steps 3 --warmup 1 $Q > $O/quick4e_${E//[=,]/_}.json 2> $O/quick4e.err || exit 6 ;;
    forcedist)
        # the N > 1 cfg-2 step (local keys, RCCL all-gather on the scan stream, device merge) at world 1
        timeout -k 10 300 python3 bench.py --force-dist --steps 50 --warmup 5 --no-cfg3 $Q > $O/forcedist.json 2> $O/forcedist.err || exit 12 ;;
    quick4)
        timeout -k 10 300 python3 bench.py --workload cfg4 --steps 3 --warmup 1 $Q > $O/quick4.json 2> $O/quick4.err || exit 6 ;;
    cfg5c:*)
        # cfg5c:N  cfg 5 at N engine contexts, 5 timed steps, no CPU baseline / PMC
        N=${S#cfg5c:}
        timeout -k 10 900 python3 bench.py --workload cfg5 --contexts $N --steps 5 --warmup 2 $Q > $O/cfg5c$N.json 2> $O/cfg5c$N.err || exit 4 ;;
    rehearse:*)
        # rehearse:N[:W]  bench.py's N > 1 path with N gloo ranks on this one GPU (tools/rehearse_multi.sh)
        R=${S#rehearse:}; N=${R%%:*}; W=cfg4; [[ $R == *:* ]] && W=${R#*:}
        bash tools/rehearse_multi.sh $TAG $N $W || exit 11 ;;
    cfg3v:*)
        # cfg3v:V  cfg 3 (30 steps) with the variant library vlib/V
        V=${S#cfg3v:}
        timeout -k 10 600 env PF_LIB_PATH=$PWD/vlib/$V/libpokec_fas.so python3 bench.py --workload cfg3 --steps 30 --warmup 5 $Q > $O/cfg3v_$V.json 2> $O/cfg3v_$V.err || exit 4 ;;
    cfg5v:*)
        # cfg5v:V  cfg 5 at one context with the variant library vlib/V
        V=${S#cfg5v:}
        timeout -k 10 900 env PF_LIB_PATH=$PWD/vlib/$V/libpokec_fas.so python3 bench.py --workload cfg5 --contexts 1 --steps 5 --warmup 2 $Q > $O/cfg5v_$V.json 2> $O/cfg5v_$V.err || exit 4 ;;
    cfg5e:*)
        # cfg5e:SETTINGS  cfg 5 at one context under PF_DEBUG=SETTINGS (e.g. chunks=6)
        E=${S#cfg5e:}
        timeout -k 10 900 env PF_DEBUG=$E python3 bench.py --workload cfg5 --contexts 1 --steps 5 --warmup 2 $Q > $O/cfg5e_${E//[=,]/_}.json 2> $O/cfg5e_${E//[=,]/_}.err || exit 4 ;;
    cfg5c1|cfg5c1:*)
        # cfg 5 at one context with the host stage clocks; cfg5c1:K runs K timed steps (default 5)
        K=5; [[ $S == cfg5c1:* ]] && K=${S#cfg5c1:}
        timeout -k 10 900 env PF_DEBUG=host_prof=1 python3 bench.py --workload cfg5 --contexts 1 --steps $K --warmup 2 $Q > $O/cfg5c1_$K.json 2> $O/cfg5c1_$K.err || exit 4 ;;
    k5t|k5t:*)
        # profiling build (K5T=1) per-phase K5 clocks; k5t:V uses vlib/V
        V=k5t; [[ $S == k5t:* ]] && V=${S#k5t:}
        timeout -k 10 300 env PF_LIB_PATH=$PWD/vlib/$V/libpokec_fas.so python3 bench.py --steps 30 --warmup 5 $Q > $O/$V.json 2> $O/$V.err || exit 7 ;;
    pmcpasses:*)
        # pmcpasses:KERNEL-REGEX  tools/pmc_passes.sh's five counter passes (TAG_KERNEL) over a short cfg-2 run
        K=${S#pmcpasses:}
        timeout -k 10 700 bash tools/pmc_passes.sh ${TAG}_$K $K || exit 8 ;;
    pmcv:*)
        # pmcv:V:C1,C2..  one counter pass over 20 cfg-2 steps with the variant library vlib/V (K5 rows only)
        R=${S#pmcv:}; V=${R%%:*}; C=${R#*:}
        timeout -s KILL 120 env PF_LIB_PATH=$PWD/vlib/$V/libpokec_fas.so rocprofv3 --pmc ${C//,/ } --kernel-include-regex fas_post -d $O/pmcv_$V -o run -- python3 bench.py --steps 20 --warmup 5 $Q > $O/pmcv_$V.json 2> $O/pmcv_$V.err || exit 8 ;;
    pmc:*)
        R=${S#pmc:}; N=${R%%:*}; C=${R#*:}
        timeout -s KILL 120 rocprofv3 --pmc ${C//,/ } -d $O/pmc_$N -o run -- python3 bench.py --steps 20 --warmup 5 $Q > $O/pmc_$N.json 2> $O/pmc_$N.err || exit 8 ;;
    ab:*)
        IFS=: read -r _ W N R AB <<< "$S"
        for ((i = 0; i < R; i++)); do
            for V in "${AB%%/*}" "${AB#*/}"; do
                E=(env)
                if [[ $V == lib=* ]]; then E+=(PF_LIB_PATH=$PWD/vlib/${V#lib=}/libpokec_fas.so)
                elif [[ $V != - ]]; then E+=(PF_DEBUG=$V); fi
                timeout -k 10 600 "${E[@]}" python3 bench.py --workload $W --steps $N --warmup 10 $Q > $O/ab.json 2> $O/ab.err || exit 13
                (echo -n "$V "; tail -1 $O/ab.json) >> $O/ab_$W.txt
            done
        done ;;
    trace:*)
        N=${S#trace:}
        timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o tr -- python3 bench.py --steps $N --warmup 5 $Q > $O/trace.json 2> $O/trace.err || exit 3 ;;
    *)
        echo "unknown step $S"; exit 9 ;;
    esac
done
echo "== done $(date +%T)"
