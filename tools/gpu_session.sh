#!/bin/bash
# One GPU-box session: GPU tests, the default bench line, a cfg2-only kernel
# trace, and the cfg5 (lreg) FETCH_SIZE / WRITE_SIZE passes.
#   bash tools/gpu_session.sh TAG [steps...]   -> gpurun_out/TAG/...
# steps: tests bench trace2 lregpmc (default: all, in that order).  A step
# that ends in a fault, abort, signal or time limit stops the session (no
# further GPU work in this call); an ordinary test failure (pytest exit 1)
# does not.  The steps that load dev builds from tools/bin/ (kab, kclk,
# ablate, gemm*) need that directory uploaded: .gpurunignore lists it (the
# round-end runs never read it), so drop that line for such a session.
R=$GRAFT_REPO_ROOT
T=${1:-sess}
shift
STEPS=${*:-tests bench trace2 lregpmc}
O=$R/gpurun_out/$T
mkdir -p $O
export TMPDIR=/tmp
step() {  # name, limit, command...
  local name=$1 lim=$2
  shift 2
  echo "[$(date +%T)] $name" >> $O/steps.log
  timeout -k 10 $lim "$@"
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" >> $O/steps.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping: $name ended with $rc" >> $O/steps.log
    exit $rc
  fi
}
for s in $STEPS; do
  case $s in
    tests)
      cd $R && step tests 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider > $O/pytest.log 2>&1 ;;
    testsp)
      # the GPU suite with passed tests' output shown (the cfg4 margin lines)
      cd $R && step testsp 900 python -u -m pytest tests -m gpu -v -rP --timeout 300 --timeout-method thread \
        -p no:cacheprovider > $O/pytest.log 2>&1 ;;
    smoke)
      cd $R && step smoke 300 python3 -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > $O/smoke.log 2>&1 ;;
    lregtests)
      cd $R && step lregtests 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider -k "sgd or lreg or golden or dot_reduce" > $O/lregtests.log 2>&1 ;;
    lregbench)
      cd $R && step lregbench 600 python3 bench.py --dot 0 --workloads lreg --cpu-baseline 0 > $O/lregbench.json 2> $O/lregbench.err ;;
    kmquick)
      # small fused-step cases first (ragged units, same-label units, all K / D shapes)
      cd $R && step kmquick 240 python -u -m pytest tests/test_gpu_parity.py -v --timeout 60 --timeout-method thread \
        -p no:cacheprovider -k "kmeans_step_same_row or kmeans_step_matches" > $O/kmquick.log 2>&1 ;;
    dottests)
      cd $R && step dottests 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider -k "dot or gemm" > $O/dottests.log 2>&1 ;;
    gemmgfl2)
      cd $R && step gemmgfl2 900 ./tools/bin/gemm_tune 32768 2 gfl2 > $O/gemmgfl2.txt 2>&1 ;;
    gemmgfl)
      cd $R && step gemmgfl 600 ./tools/bin/gemm_tune 32768 2 gfl > $O/gemmgfl.txt 2>&1 ;;
    kmdiag)
      cd $R && step kmdiag 150 python3 -u tools/km_diag.py 1200000 > $O/kmdiag.log 2>&1 ;;
    kpprof)
      # per-segment cycles of the fused step (tools/kp_prof.sh build)
      cd $R && step kpprof 240 python3 tools/kp_prof.py 100000000 > $O/kpprof.txt 2>&1 ;;
    ablate)
      # k_kmeans_pp ablation builds (tools/kp_ablate.sh), kernel-traced one by one
      for f in $R/tools/bin/libspx_abl_*.so; do
        n=$(basename $f .so)
        cd /tmp && step $n 120 rocprofv3 --kernel-trace --stats -d $O/abl/$n -o p --output-format csv \
          -- python3 $R/tools/km_step_once.py 100000000 3 step $f > $O/$n.log 2>&1
      done ;;
    kmcounts)
      cd $R && step kmcounts 120 python3 tools/km_counts.py 100000000 > $O/kmcounts.txt 2>&1 && \
        step kmcounts_first 120 python3 tools/km_counts.py 100000000 first >> $O/kmcounts.txt 2>&1 ;;
    kmfit)
      cd $R && step kmfit 240 python3 tools/km_fit_timing.py 100000000 2 $KMFIT_OLD > $O/kmfit.txt 2>&1 ;;
    dotbench)
      cd $R && step dotbench 600 python3 bench.py --workloads 0 --cpu-baseline 0 --steps 2 --warmup 1 > $O/dotbench.json 2> $O/dotbench.err ;;
    kmtests)
      cd $R && step kmtests 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread \
        -p no:cacheprovider -k "kmeans" > $O/kmtests.log 2>&1 ;;
    kmbench)
      cd $R && step kmbench 600 python3 bench.py --dot 0 --workloads kmeans --cpu-baseline 0 --steps 2 --warmup 1 \
        > $O/kmbench.json 2> $O/kmbench.err ;;
    kmtrace)
      cd /tmp && step kmtrace 300 rocprofv3 --kernel-trace --stats -d $O/kmtrace -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads kmeans --cpu-baseline 0 --steps 2 --warmup 1 > $O/kmtrace.log 2>&1 ;;
    kstrace)
      # kernel trace of the fused step alone (tools/km_step_once.py at cfg3, second-iteration centres)
      cd /tmp && step kstrace 300 rocprofv3 --kernel-trace --stats -d $O/kstrace -o p --output-format csv \
        -- python3 $R/tools/km_step_once.py 100000000 5 > $O/kstrace.log 2>&1 ;;
    kftrace)
      # the same on first-iteration centres (the first K points: skewed labels, more add rounds)
      cd /tmp && step kftrace 300 rocprofv3 --kernel-trace --stats -d $O/kftrace -o p --output-format csv \
        -- python3 $R/tools/km_step_once.py 100000000 5 first > $O/kftrace.log 2>&1 ;;
    kab)
      # A/B of libspx builds on one box: the fused step under a kernel trace,
      # each build twice in alternation (KAB: names of tools/bin/libspx_NAME.so,
      # 'product' = spartan_amd/libspx.so); the fused kernel's time per call
      # is in $O/kab_NAME_i/p_kernel_stats.csv
      for i in 1 2; do
        for v in ${KAB:-base product}; do
          lib=$R/tools/bin/libspx_$v.so; [ $v = product ] && lib=$R/spartan_amd/libspx.so
          cd /tmp && step kab_${v}_$i 120 rocprofv3 --kernel-trace --stats -d $O/kab_${v}_$i -o p --output-format csv \
            -- python3 $R/tools/km_step_once.py 100000000 5 ${KAB_MODE:-step} $lib > $O/kab_${v}_$i.log 2>&1
        done
      done ;;
    kclk)
      # clock and wave-state counters of the fused step per build (KAB names)
      for v in ${KAB:-product}; do
        lib=$R/tools/bin/libspx_$v.so; [ $v = product ] && lib=$R/spartan_amd/libspx.so
        cd /tmp && step kclk_$v 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY \
          SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU \
          -d $O/kclk_$v -o p --output-format csv -- python3 $R/tools/km_step_once.py 100000000 2 step $lib > $O/kclk_$v.log 2>&1
      done ;;
    kundtrace)
      cd /tmp && step kundtrace 300 rocprofv3 --kernel-trace --stats -d $O/kundtrace -o p --output-format csv \
        -- python3 $R/tools/km_und.py 100000000 > $O/kundtrace.log 2>&1 ;;
    kfspmc)
      # counter passes over the fused k-means step (one group per pass: the box rejects overfull groups)
      cd /tmp
      step kfs_a 120 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE \
        -d $O/kfs_a -o p --output-format csv -- python3 $R/tools/km_step_once.py 100000000 2 > $O/kfs_a.log 2>&1
      step kfs_b 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM GRBM_GUI_ACTIVE \
        -d $O/kfs_b -o p --output-format csv -- python3 $R/tools/km_step_once.py 100000000 2 > $O/kfs_b.log 2>&1 ;;
    kfsmem)
      # vector-memory counters over the fused step: product build, then the
      # coalesced-load ablation if built (tools/kp_ablate.sh coal)
      cd /tmp
      for v in product coal; do
        lib=""; [ $v = coal ] && lib=$R/tools/bin/libspx_abl_coal.so
        [ $v = coal ] && [ ! -f "$lib" ] && continue
        step kfsmem_a_$v 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum \
          TCP_PENDING_STALL_CYCLES_sum TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE \
          -d $O/kfsmem_a_$v -o p --output-format csv -- python3 $R/tools/km_step_once.py 100000000 2 step $lib > $O/kfsmem_a_$v.log 2>&1
        step kfsmem_b_$v 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum \
          TCP_TD_TCP_STALL_CYCLES_sum TD_TC_STALL_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE \
          -d $O/kfsmem_b_$v -o p --output-format csv -- python3 $R/tools/km_step_once.py 100000000 2 step $lib > $O/kfsmem_b_$v.log 2>&1
      done ;;
    kfslds)
      # LDS counters over the fused k-means step (bank conflicts vs all LDS-array cycles)
      cd /tmp
      step kfs_lds 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVES GRBM_GUI_ACTIVE \
        -d $O/kfs_lds -o p --output-format csv -- python3 $R/tools/km_step_once.py 100000000 2 > $O/kfs_lds.log 2>&1 ;;
    lregsweep)
      cd $R && step lregsweep 600 python3 tools/lreg_sweep.py 100000000 10 2 > $O/lregsweep.txt 2>&1 ;;
    lregtune)
      cd $R && step lregtune 300 ./tools/bin/lreg_tune 100000000 3 > $O/lregtune.txt 2>&1 ;;
    gemmseg2)
      cd $R && step gemmseg2 600 ./tools/bin/gemm_tune 32768 2 seg2 > $O/gemmseg2.txt 2>&1 ;;
    gemmseg)
      cd $R && step gemmseg 600 ./tools/bin/gemm_tune 32768 2 seg > $O/gemmseg.txt 2>&1 ;;
    bench)
      cd $R && step bench 600 python3 bench.py > $O/bench.json 2> $O/bench.err ;;
    trace2)
      cd /tmp && step trace2 300 rocprofv3 --kernel-trace --stats -d $O/trace2 -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads 0 --cpu-baseline 0 --steps 20 --warmup 5 > $O/trace2.log 2>&1 ;;
    benchtrace)
      # the default bench (minus the CPU legs) under a kernel trace: its JSON
      # line and the trace come from the SAME run (profiles/ roofline check)
      cd /tmp && step benchtrace 600 rocprofv3 --kernel-trace --stats -d $O/benchtrace -o p --output-format csv \
        -- python3 $R/bench.py --cpu-baseline 0 > $O/benchtrace.json 2> $O/benchtrace.err ;;
    traceall)
      cd /tmp && step traceall 600 rocprofv3 --kernel-trace --stats -d $O/traceall -o p --output-format csv \
        -- python3 $R/bench.py --cpu-baseline 0 --steps 5 --warmup 1 > $O/traceall.log 2>&1 ;;
    trace5)
      cd /tmp && step trace5 300 rocprofv3 --kernel-trace --stats -d $O/trace5 -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads lreg --cpu-baseline 0 --steps 2 --warmup 1 > $O/trace5.log 2>&1 ;;
    lregpmc)
      cd /tmp && step lregf 300 rocprofv3 --pmc FETCH_SIZE -d $O/lregf -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads lreg --cpu-baseline 0 --steps 2 --warmup 1 > $O/lregf.log 2>&1
      cd /tmp && step lregw 300 rocprofv3 --pmc WRITE_SIZE -d $O/lregw -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads lreg --cpu-baseline 0 --steps 2 --warmup 1 > $O/lregw.log 2>&1 ;;
    cfg2pmc)
      cd /tmp && step c2f 300 rocprofv3 --pmc FETCH_SIZE -d $O/c2f -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads 0 --cpu-baseline 0 --steps 3 --warmup 1 > $O/c2f.log 2>&1
      cd /tmp && step c2w 300 rocprofv3 --pmc WRITE_SIZE -d $O/c2w -o p --output-format csv \
        -- python3 $R/bench.py --dot 0 --workloads 0 --cpu-baseline 0 --steps 3 --warmup 1 > $O/c2w.log 2>&1 ;;
    kmpmc)
      cd /tmp && step kmf 300 rocprofv3 --pmc FETCH_SIZE -d $O/kmf -o p --output-format csv \
        -- python3 $R/tools/km_step_once.py 100000000 2 > $O/kmf.log 2>&1
      cd /tmp && step kmw 300 rocprofv3 --pmc WRITE_SIZE -d $O/kmw -o p --output-format csv \
        -- python3 $R/tools/km_step_once.py 100000000 2 > $O/kmw.log 2>&1 ;;
    *)
      # anything else: a python script under tools/ with its arguments joined by ':'
      cd $R && step "$s" 600 python3 ${s//:/ } > $O/$(echo "$s" | tr '/:' '__').log 2>&1 ;;
  esac
done
echo "[$(date +%T)] session done" | tee -a $O/steps.log
