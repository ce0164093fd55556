#!/bin/bash
# Round-6 GPU runs (gpurun): `scripts/gpu_r06.sh STEP...`, each step under its own limit,
# stopping at the first failure.
#   full     tests/test_gpu_fullsize.py (whole-stream digests at 64/1M and 256/10M)
#   gpu      the whole pytest -m gpu suite
#   bench    the default bench line (256/10M) -> gpurun_out/r06/bench.json
#   mc       bench.py --workload mc -> gpurun_out/r06/bench_mc.json
#   prof     rocprofv3 kernel stats of the default bench -> gpurun_out/r06/prof
#   profmc   rocprofv3 kernel stats of the mc bench -> gpurun_out/r06/profmc
#   smoke    __graft_entry__.smoke()
#   fallback the hand-off fallback and RCCL world-1 exchange tests
#   emulate  the one-hashgraph split emulated part by part (256/10M, 2/4/8 parts)
#   configs  16/100k, 32/1M, 64/1M, 128/1M bench lines
#   pmc      FETCH_SIZE / WRITE_SIZE passes -> profiles/r06/pmc_traffic.json (the bench's roofline traffic)
#   diag     SQ / TCC / LDS counter passes at 256/2M
#   gap      microbenchmarks: launch_gap (stream launches vs a HIP graph), granule_hop (hand-off floor)
#   ab       same-box A/B: build/ab/libhge_head.so (the last commit's engine), build/ab/libhge_alt.so
#            (a variant, when present) and this tree's
#   abfd     A/B of the rounds kernel without the window's FD rows in LDS (HGE_DIR_NOFD)
#   core     parity, wide, golden and replay-path GPU tests
#   online   per-call profile of the online path (16/100k, 256 prefix)
#   onprof   rocprofv3 kernel stats and SQ counters of 400 online calls at 256 participants
#   stamps   the batch engine's per-section cycle stamps (HGB_STAMPS)
#   onphase  online calls at 16, 64 and 256 participants with HGE_HOST_PHASES (host time split)
#   gapargs / gapcopies  launch_gap modes: argument size, small stream copies vs zero-copy
#   mcg      config 5 at GRAPHS="..." graphs per GPU
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 9
mkdir -p gpurun_out/r06
PYT="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
for s in "$@"; do
  echo "== $s $(date +%T)"
  case "$s" in
    full) timeout -k 10 400 $PYT -m gpu tests/test_gpu_fullsize.py > gpurun_out/r06/full.log 2>&1 || { tail -30 gpurun_out/r06/full.log; exit 1; }
          tail -3 gpurun_out/r06/full.log ;;
    gpu) timeout -k 10 900 $PYT -m gpu tests > gpurun_out/r06/gpu.log 2>&1 || { tail -40 gpurun_out/r06/gpu.log; exit 1; }
         tail -3 gpurun_out/r06/gpu.log ;;
    batch) timeout -k 10 600 $PYT -m gpu tests/test_gpu_batch.py > gpurun_out/r06/batch.log 2>&1 || { tail -60 gpurun_out/r06/batch.log; exit 1; }
         tail -3 gpurun_out/r06/batch.log ;;
    fallback) timeout -k 10 400 $PYT -m gpu tests/test_gpu_wide.py tests/test_gpu_split.py -k "handoff or nccl_world or stall" > gpurun_out/r06/fallback.log 2>&1 || { tail -40 gpurun_out/r06/fallback.log; exit 1; }
         tail -3 gpurun_out/r06/fallback.log ;;
    stamps) HGB_STAMPS=1 timeout -k 10 300 python -u bench.py --workload mc --no-cpu-baseline --steps 2 --warmup 1 --ramp-s 0 > gpurun_out/r06/stamps.json 2> gpurun_out/r06/stamps.err || { tail -20 gpurun_out/r06/stamps.err; exit 2; }
         grep "hgb stamps" gpurun_out/r06/stamps.err | tail -1 ;;
    online) timeout -k 10 300 python -u scripts/analysis/online_profile.py 16 100000 16 2000 > gpurun_out/r06/online16.json 2> gpurun_out/r06/online16.err || { tail -20 gpurun_out/r06/online16.err; exit 2; }
         timeout -k 10 300 python -u scripts/analysis/online_profile.py 256 600000 256 800 > gpurun_out/r06/online256.json 2> gpurun_out/r06/online256.err || { tail -20 gpurun_out/r06/online256.err; exit 2; }
         head -12 gpurun_out/r06/online16.json ;;
    core) timeout -k 10 600 $PYT -m gpu tests/test_gpu_parity.py tests/test_gpu_wide.py tests/test_gpu_golden.py tests/test_gpu_replay_paths.py tests/test_gpu_reference.py > gpurun_out/r06/core.log 2>&1 || { tail -40 gpurun_out/r06/core.log; exit 1; }
         tail -3 gpurun_out/r06/core.log ;;
    emulate) timeout -k 10 600 python -u scripts/analysis/split_emulate.py 256 10000000 2 4 8 > gpurun_out/r06/emulate.log 2>&1 || { tail -20 gpurun_out/r06/emulate.log; exit 3; }
         grep -E "unsplit|max part" gpurun_out/r06/emulate.log ;;
    configs) for NE in "16 100000" "32 1000000" "64 1000000" "128 1000000"; do
           set -- $NE
           timeout -k 10 300 python -u bench.py --participants $1 --events $2 --no-secondary --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/r06/n$1_e$2.json 2> gpurun_out/r06/n$1_e$2.err || { tail -20 gpurun_out/r06/n$1_e$2.err; exit 1; }
           python -c "
import json
d=json.loads(open('gpurun_out/r06/n$1_e$2.json').read().strip().splitlines()[-1])
print('$1/$2', round(d['value']/1e6,2), d['ms_per_step'], d['parity'][:120])"
         done ;;
    gap) timeout -k 10 120 ./build/launch_gap 32 2000 > gpurun_out/r06/launch_gap.json && timeout -k 10 120 ./build/launch_gap 16 2000 >> gpurun_out/r06/launch_gap.json || exit 5
         timeout -k 10 120 ./build/granule_hop 256 4000 > gpurun_out/r06/granule_hop.json || exit 5
         cat gpurun_out/r06/launch_gap.json gpurun_out/r06/granule_hop.json ;;
    gapargs) timeout -k 10 120 ./build/launch_gap args 20 2000 > gpurun_out/r06/launch_args.json && timeout -k 10 120 ./build/launch_gap args 8 2000 >> gpurun_out/r06/launch_args.json || exit 5
         cat gpurun_out/r06/launch_args.json ;;
    gapcopies) timeout -k 10 120 ./build/launch_gap copies 16 2000 > gpurun_out/r06/launch_copies.json && timeout -k 10 120 ./build/launch_gap copies 8 2000 >> gpurun_out/r06/launch_copies.json || exit 5
         cat gpurun_out/r06/launch_copies.json ;;
    onphase) for NE in "16 100000 16 3000" "64 1000000 64 2000" "256 600000 256 600"; do
           HGE_HOST_PHASES=1 timeout -k 10 300 python -u scripts/analysis/online_profile.py $NE > gpurun_out/r06/onphase.json 2> gpurun_out/r06/onphase.err || { tail -20 gpurun_out/r06/onphase.err; exit 2; }
           python -c "import json; d=json.load(open('gpurun_out/r06/onphase.json')); print('$NE', d['plain']['p50_us'], d['plain']['mean_us'], d['profiled']['launches_per_call'])"
           grep hge_host_phases gpurun_out/r06/onphase.err | head -1
         done ;;
    ab16) for v in head new head new; do
           case $v in head) export HGE_LIB=build/ab/libhge_head.so ;; *) unset HGE_LIB ;; esac
           for NE in ${AB_CONFIGS:-16:100000 32:1000000}; do
             set -- ${NE/:/ }
             timeout -k 10 300 python -u bench.py --participants $1 --events $2 --no-secondary --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/r06/ab16_${v}_$1.json 2> gpurun_out/r06/ab16_${v}_$1.err || { tail -5 gpurun_out/r06/ab16_${v}_$1.err; exit 2; }
             python -c "
import json
d=json.loads(open('gpurun_out/r06/ab16_${v}_$1.json').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$v', '$1/$2', round(d['value']/1e6,2), d['ms_per_step'], {n: round(k[n],3) for n in k if 'fame' in n}, d['parity'][:30])"
           done
         done; unset HGE_LIB ;;
    pmc) bash scripts/gpu_pmc.sh r06/pmc || exit 6 ;;
    diag) bash scripts/gpu_pmc_diag.sh r06/diag && bash scripts/gpu_pmc_lds.sh r06/lds || exit 6 ;;
    onprof) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/onprof -o run -- python3 -u scripts/analysis/online_profile.py 256 600000 256 400 > gpurun_out/r06/onprof.log 2>&1 || { tail -20 gpurun_out/r06/onprof.log; exit 7; }
         timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d gpurun_out/r06/onpmc -o pmc -- python3 -u scripts/analysis/online_profile.py 256 600000 256 400 > gpurun_out/r06/onpmc.log 2>&1 || { tail -20 gpurun_out/r06/onpmc.log; exit 7; }
         find gpurun_out/r06 -name "*.db" -delete; find gpurun_out/r06/onpmc gpurun_out/r06/onprof -name "*kernel_trace.csv" -delete
         find gpurun_out/r06/onprof -name "*kernel_stats.csv" | head -1 | xargs head -20 ;;
    segdbg) HGE_STAMPS=1 HGE_SEG_DEBUG=1 timeout -k 10 300 python3 -u scripts/analysis/online_profile.py 256 600000 256 300 > gpurun_out/r06/segdbg.json 2> gpurun_out/r06/segdbg.err || { tail -5 gpurun_out/r06/segdbg.err; exit 7; }
         grep "hge seg" gpurun_out/r06/segdbg.err | sort | uniq -c | sort -rn | head -8; grep "hge theta" gpurun_out/r06/segdbg.err | tail -3 ;;
    abfd) for v in 0 1 0 1; do
           if [ $v = 1 ]; then export HGE_DIR_NOFD=1; else unset HGE_DIR_NOFD; fi
           timeout -k 10 300 python -u bench.py --no-secondary --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r06/abfd_$v.json 2> gpurun_out/r06/abfd_$v.err || { tail -5 gpurun_out/r06/abfd_$v.err; exit 2; }
           python -c "
import json
d=json.loads(open('gpurun_out/r06/abfd_$v.json').read().strip().splitlines()[-1])
print('nofd=$v', round(d['value']/1e6,2), d['ms_per_step'], d['kernels_ms_per_replay']['k_rounds_direct'], d['parity'][:40])"
         done; unset HGE_DIR_NOFD ;;
    ab) vs="head new head new"; [ -f build/ab/libhge_alt.so ] && vs="head alt new head alt new"
         for v in $vs; do
           case $v in head) export HGE_LIB=build/ab/libhge_head.so ;; alt) export HGE_LIB=build/ab/libhge_alt.so ;; *) unset HGE_LIB ;; esac
           timeout -k 10 300 python -u bench.py --no-secondary --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r06/ab_$v.json 2> gpurun_out/r06/ab_$v.err || { tail -5 gpurun_out/r06/ab_$v.err; exit 2; }
           python -c "
import json
d=json.loads(open('gpurun_out/r06/ab_$v.json').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$v', round(d['value']/1e6,2), d['ms_per_step'], {n: k[n] for n in k if 'transpose' in n or 'runs' in n or 'rounds_direct' in n}, d['parity'][:40])"
         done; unset HGE_LIB ;;
    mcgpu) timeout -k 10 600 $PYT -m gpu tests/test_gpu_mc.py tests/test_gpu_batch.py > gpurun_out/r06/mcgpu.log 2>&1 || { tail -40 gpurun_out/r06/mcgpu.log; exit 1; }
         tail -3 gpurun_out/r06/mcgpu.log ;;
    bench) timeout -k 10 600 python -u bench.py > gpurun_out/r06/bench.json 2> gpurun_out/r06/bench.err || { tail -20 gpurun_out/r06/bench.err; exit 2; }
           python -c "
import json
d=json.loads(open('gpurun_out/r06/bench.json').read().strip().splitlines()[-1])
print(round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['frac']); print(d['parity'])
print(d['kernels_ms_per_replay'])" ;;
    mc) timeout -k 10 600 python -u bench.py --workload mc > gpurun_out/r06/bench_mc.json 2> gpurun_out/r06/bench_mc.err || { tail -20 gpurun_out/r06/bench_mc.err; exit 2; }
        python -c "
import json
d=json.loads(open('gpurun_out/r06/bench_mc.json').read().strip().splitlines()[-1])
print(round(d['value']/1e6,2), d['ms_per_step'], d['roofline']['frac']); print(d['parity']); print(d['cpu_baseline'])
print(d['kernels_ms_per_replay'])" ;;
    mc128) timeout -k 10 600 python -u bench.py --workload mc --graphs 128 --no-cpu-baseline > gpurun_out/r06/bench_mc128.json 2> gpurun_out/r06/bench_mc128.err || { tail -20 gpurun_out/r06/bench_mc128.err; exit 2; }
        python -c "
import json
d=json.loads(open('gpurun_out/r06/bench_mc128.json').read().strip().splitlines()[-1])
print('mc128', round(d['value']/1e6,2), d['ms_per_step'], d['parity']); print(d['kernels_ms_per_replay'])" ;;
    stamps128) HGB_STAMPS=1 timeout -k 10 300 python -u bench.py --workload mc --graphs 128 --no-cpu-baseline --steps 2 --warmup 1 --ramp-s 0 > gpurun_out/r06/stamps128.json 2> gpurun_out/r06/stamps128.err || { tail -20 gpurun_out/r06/stamps128.err; exit 2; }
         grep "hgb stamps" gpurun_out/r06/stamps128.err | tail -1 ;;
    trace) timeout -k 10 600 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r06/trace -o run -- python -u bench.py --no-secondary --no-cpu-baseline --steps 1 --warmup 0 --ramp-s 0 --profile-steps 1 > gpurun_out/r06/trace.log 2>&1 || { tail -20 gpurun_out/r06/trace.log; exit 3; }
          python scripts/analysis/gaps.py gpurun_out/r06/trace > gpurun_out/r06/gaps.txt && head -40 gpurun_out/r06/gaps.txt
          find gpurun_out/r06/trace -name "*.db" -delete ;;
    abenv) for v in 0 1 0 1; do
           if [ $v = 1 ]; then export $ABVAR=1; else unset $ABVAR; fi
           timeout -k 10 300 python -u bench.py --no-secondary --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r06/ab_${ABVAR}_$v.json 2> gpurun_out/r06/ab_${ABVAR}_$v.err || { tail -5 gpurun_out/r06/ab_${ABVAR}_$v.err; exit 2; }
           python -c "
import json
d=json.loads(open('gpurun_out/r06/ab_${ABVAR}_$v.json').read().strip().splitlines()[-1])
k=d['kernels_ms_per_replay']
print('$ABVAR=$v', round(d['value']/1e6,2), d['ms_per_step'], {n: k[n] for n in k if 'median' in n or 'rows_runs' in n or 'transpose' in n or 'rounds_direct' in n}, d['parity'][:60])"
         done; unset $ABVAR ;;
    mcg) for G in $GRAPHS; do
           timeout -k 10 300 python -u bench.py --workload mc --graphs $G --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/r06/bench_mc$G.json 2> gpurun_out/r06/bench_mc$G.err || { tail -20 gpurun_out/r06/bench_mc$G.err; exit 2; }
           python -c "
import json
d=json.loads(open('gpurun_out/r06/bench_mc$G.json').read().strip().splitlines()[-1])
print('mc$G', round(d['value']/1e6,2), d['ms_per_step'], d['config']['ordered_per_step'], d['parity'][:50]); print(d['kernels_ms_per_replay'])"
         done ;;
    prof) timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/prof -o run -- python -u bench.py --no-secondary --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r06/prof.log 2>&1 || { tail -20 gpurun_out/r06/prof.log; exit 3; }
          find gpurun_out/r06/prof -name "*kernel_trace.csv" -delete; find gpurun_out/r06/prof -name "*kernel_stats.csv" | head -1 | xargs head -12 ;;
    profmc) timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06/profmc -o run -- python -u bench.py --workload mc --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/r06/profmc.log 2>&1 || { tail -20 gpurun_out/r06/profmc.log; exit 3; }
            find gpurun_out/r06/profmc -name "*kernel_trace.csv" -delete; find gpurun_out/r06/profmc -name "*kernel_stats.csv" | head -1 | xargs head -20 ;;
    smoke) timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r06/smoke.log 2>&1 || { tail -20 gpurun_out/r06/smoke.log; exit 4; }
           tail -1 gpurun_out/r06/smoke.log ;;
    *) echo "unknown step $s"; exit 8 ;;
  esac
done
echo "== done $(date +%T)"
