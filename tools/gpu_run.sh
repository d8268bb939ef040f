#!/bin/bash
# GPU session driver: each step under its own time limit; a step that times out, aborts or faults
# (exit 124 / 134 / 137 / 139) ends the session (nothing more runs on the GPU), a failing test does not.
# Steps on the development library (doavar, fixcount, k1cap, mall) need `make -C radar-slam_amd/csrc dev` first, the
# ab steps `tools/build_ab.sh <commit>`.
# usage: bash tools/gpu_run.sh TAG step...   steps: tests | testsall | fixcount | smoke | bench | benchq | doactr | prof | ab | k1cap
set -u
TAG=$1; shift
mkdir -p gpurun_out
export TMPDIR=/tmp
stop() { echo "step $1 ended with $2: stopping"; exit $2; }
run() {  # name seconds cmd...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "$name rc $rc"
  case $rc in 124|134|137|139) stop "$name" $rc;; esac
}
for step in "$@"; do
  case $step in
    tests) run tests 560 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread ;;
    tdoa) run tdoa 400 python -u -m pytest tests/test_gpu_doa_exact.py tests/test_gpu_chain.py tests/test_gpu_sweep.py tests/test_gpu_spectrum.py -x -q --timeout 150 --timeout-method thread ;;
    tsel) run tsel 400 python -u -m pytest tests/test_gpu_dbmap.py tests/test_gpu_doa_exact.py tests/test_gpu_chain.py tests/test_gpu_scheduling.py tests/test_gpu_pipelined.py -x -q --timeout 150 --timeout-method thread ;;
    testsall) run testsall 600 python -u -m pytest tests -m gpu -q --maxfail 12 --timeout 150 --timeout-method thread ;;
    doavar) RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so run doavar 300 python -u tools/doa_var_time.py 0
      RSL_LIBRARY=radar-slam_amd/lib/librsl_ab.so run doavar_ab 200 python -u tools/doa_var_time.py 0 ;;
    doaab)  # DoA scan + fixup alone, product vs radar-slam_amd/lib/librsl_ab.so (tools/build_ab.sh), 2 rounds
      for r in 1 2; do
        RSL_LIBRARY=radar-slam_amd/lib/librsl_ab.so run doaab_old$r 200 python -u tools/doa_var_time.py 0
        run doaab_new$r 200 python -u tools/doa_var_time.py 0
      done ;;
    dgrid)  # DoA scan as a persistent share (dev library, RSL_DOA_GRID workgroups): pipelined bench + standalone DoA
      for g in 0 256 512 768; do
        RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so RSL_DOA_GRID=$g run dgrid_b$g 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra
        RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so RSL_DOA_GRID=$g run dgrid_d$g 200 python -u tools/doa_var_time.py 0
      done
      python3 tools/ab_summary.py gpurun_out/${TAG}_dgrid_b*.log ;;
    pipe)  # pipelined two-stream step vs one stream (--pipeline 0), 2 rounds
      for r in 1 2; do
        run pipe1_$r 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra
        run pipe0_$r 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra --pipeline 0
      done
      python3 tools/ab_summary.py gpurun_out/${TAG}_pipe*.log ;;
    prio)  # stream priorities of the pipelined halves (RSL_BENCH_PRIO front:back), 2 rounds
      run prio_range 60 python -c "import torch; print(torch.cuda.Stream.priority_range())"
      for r in 1 2; do
        for pr in 0:0 -1:0 0:-1; do RSL_BENCH_PRIO=$pr run prio${pr/:/_}_$r 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra; done
      done
      cat gpurun_out/${TAG}_prio_range.log
      for f in gpurun_out/${TAG}_prio*_?.log; do python3 -c "
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')][-1]; d=json.loads(l)
print(sys.argv[1], round(d['value']), 'fft live', round(d['roofline']['frac'],3), 'doa live', round(d['roofline_doa']['frac'],3))" $f; done ;;
    cfg5f)  # configs[4] shape at 100 / 200 / 400 frames per step
      for f in 100 200 400; do run cfg5f$f 300 python -u bench.py --config cfg5 --no-cpu-baseline --no-pcie --no-extra --frames-per-step $f; done
      python3 tools/ab_summary.py gpurun_out/${TAG}_cfg5f*.log ;;
    cfg2f)  # cfg2 at 2000 / 4000 frames per step, 2 rounds
      for r in 1 2; do for f in 2000 4000; do run cfg2f${f}_$r 300 python -u bench.py --no-cpu-baseline --no-pcie --no-extra --frames-per-step $f; done; done
      python3 tools/ab_summary.py gpurun_out/${TAG}_cfg2f*.log ;;
    fixcount5) CFG=cfg5 RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so run fixcount5 300 python -u tools/doa_fix_count.py ;;
    place)  # compaction / offsets placement in the pipelined step (RSL_BENCH_EMIT_BACK 0 / 1 / 2), 2 rounds
      for r in 1 2; do for p in 0 1 2; do RSL_BENCH_EMIT_BACK=$p run place${p}_$r 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra; done; done
      python3 tools/ab_summary.py gpurun_out/${TAG}_place*.log ;;
    k1align) run k1align 300 python -u tools/k1_align.py ;;
    bound) RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so run bound 300 python -u tools/doa_bound_study.py ;;
    fixcount) RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so run fixcount 200 python -u tools/doa_fix_count.py ;;
    probe)  # hipEvent semantics (tools/event_probe.hip), alone and under the kernel trace
      run probe 60 ./tools/event_probe
      run probe_trace 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_probe_trace -o t -- ./tools/event_probe ;;
    ab3)  # product vs librsl_ab1.so vs librsl_ab.so (tools/build_ab.sh), 2 rounds, one box
      for r in 1 2; do
        RSL_LIBRARY=radar-slam_amd/lib/librsl_ab.so run ab3_old$r 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra
        RSL_LIBRARY=radar-slam_amd/lib/librsl_ab1.so run ab3_mid$r 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra
        run ab3_new$r 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra
      done
      python3 tools/ab_summary.py gpurun_out/${TAG}_ab3_*.log ;;
    ddctr) OUT=gpurun_out/${TAG}_ddctr run ddctr 400 bash tools/dd_counters.sh ;;
    ddctr5) CFG=cfg5 OUT=gpurun_out/${TAG}_ddctr5 run ddctr5 400 bash tools/dd_counters.sh ;;
    cfg5ab)  # configs[4] shape: packed register-form K1 / K2 (product) vs the c64 LDS kernels (dev library, RSL_WORK_C64=1)
      for r in 1 2; do
        RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so RSL_WORK_C64=1 run cfg5ab_old$r 200 python -u bench.py --config cfg5 --no-cpu-baseline
        run cfg5ab_new$r 200 python -u bench.py --config cfg5 --no-cpu-baseline
      done
      python3 tools/ab_summary.py gpurun_out/${TAG}_cfg5ab_*.log ;;
    cfg5abl) CFG=cfg5 C64=0 RF_LIST=0,2,3 DD_LIST=0,6,7,8 RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so run cfg5abl 200 python -u tools/fft_ablation.py ;;
    ab5)  # configs[4] shape: product vs radar-slam_amd/lib/librsl_ab.so (tools/build_ab.sh), 2 rounds
      for r in 1 2; do
        RSL_LIBRARY=radar-slam_amd/lib/librsl_ab.so run ab5_old$r 200 python -u bench.py --config cfg5 --no-cpu-baseline
        run ab5_new$r 200 python -u bench.py --config cfg5 --no-cpu-baseline
      done
      python3 tools/ab_summary.py gpurun_out/${TAG}_ab5_*.log ;;
    cfg1abl) CFG=cfg1 ONLY0=1 RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so run cfg1abl 200 python -u tools/fft_ablation.py ;;
    serialprof)  # kernel trace of the one-stream chain (standalone per-kernel times)
      run serialprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_serial -o t -- python3 bench.py --pipeline 0 --no-cpu-baseline --no-pcie --no-extra ;;
    cfg5prof) run cfg5prof 600 bash tools/profile_cfg5.sh "$TAG" ;;
    specprof) run specprof 600 bash tools/profile_spectrum.sh "$TAG" ;;
    hash)  # chain output hashes, product vs radar-slam_amd/lib/librsl_ab.so, cfg1 / cfg2 / cfg5
      for c in cfg1 cfg2 cfg5; do
        CFG=$c F=40 run hash_new_$c 120 python -u tools/chain_hash.py
        CFG=$c F=40 RSL_LIBRARY=radar-slam_amd/lib/librsl_ab.so run hash_old_$c 120 python -u tools/chain_hash.py
      done
      for c in cfg1 cfg2 cfg5; do tail -1 gpurun_out/${TAG}_hash_new_$c.log; tail -1 gpurun_out/${TAG}_hash_old_$c.log; done ;;
    tve)  # live per-kernel time: rocprofv3 kernel trace and the bench's hipEvent spans of the same run
      run tve_trace 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_tve -o trace -- python3 bench.py --no-cpu-baseline --no-pcie --no-extra
      python3 tools/trace_vs_events.py $(find gpurun_out/${TAG}_tve -name '*kernel_trace.csv' | head -1) gpurun_out/${TAG}_tve_trace.log > gpurun_out/${TAG}_tve_cmp.log 2>&1; cat gpurun_out/${TAG}_tve_cmp.log ;;
    transient) run transient 120 python -u tools/transient_row.py ;;
    smoke) run smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 400 python -u bench.py ;;
    benchq) run benchq 300 python -u bench.py --no-cpu-baseline --no-pcie --no-extra ;;
    doactr) F=1000 REPS=3 run doactr 400 bash tools/doa_counters.sh ;;
    prof) run prof 900 bash tools/profile.sh "$TAG" ;;
    ab)  # product library vs radar-slam_amd/lib/librsl_ab.so (tools/build_ab.sh), 2 rounds, one box
      for r in 1 2; do
        RSL_LIBRARY=radar-slam_amd/lib/librsl_ab.so run ab_old$r 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra
        run ab_new$r 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra
      done
      python3 tools/ab_summary.py gpurun_out/${TAG}_ab_*.log ;;
    k1cap)  # resident K1 workgroups per CU capped (dev library, RSL_K1_WG_PER_CU): room for the back stream
      for r in 1 2; do
        for n in 0 2; do RSL_LIBRARY=radar-slam_amd/lib/librsl_dev.so RSL_K1_WG_PER_CU=$n run k1cap${n}_$r 200 python -u bench.py --no-cpu-baseline --no-pcie --no-extra; done
      done
      python3 tools/ab_summary.py gpurun_out/${TAG}_k1cap*.log ;;
  esac
done
