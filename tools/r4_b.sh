#!/bin/bash
# round-4 A/B step: parity tests on the walk variants (var 7 scan cascade, 8 per-query tile masks,
# 9 both), then alternating bench runs: cfg3 (walk variants, radix vs counting query sort), cfg4
# (shared chain thresholds, fixed-width chain motion kernel), cfg5 (radius walk at 7 / 8 waves)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out=gpurun_out/r4b; mkdir -p "$out"
P=${PART:-1}  # 1: walk variants (cfg3); 2: 16-bit rows (cfg4, cfg5k, cfg3, cfg5); 3: radius variants; 5: chain prefetch
rc_ok() { case $1 in 0) ;; 124|134|137|139) exit 1;; *) echo "$2 failed";; esac; }
if [ "$P" = 1 ]; then
T="tests/test_gpu_nn.py tests/test_gpu_cull.py"
for v in ${VARS:-7 8 9 12}; do
  OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var$v.so timeout -k 10 300 python -u -m pytest $T -m gpu -x -q --timeout 200 \
      --timeout-method thread > "$out/pytest_v$v.log" 2>&1
  rc=$?; echo "var$v: $(tail -1 "$out/pytest_v$v.log")"; rc_ok $rc var$v
done
bash tools/ab_env.sh cfg3 "--workload cfg3" 2 - VAR=7 VAR=8 VAR=9 VAR=12 OMPL_GPU_QSORT=0 || exit 1
fi
if [ "$P" = 2 ]; then  # the 16-bit rows: chain cull (default on), SE3 kNN and radius walks (A/B)
TESTS_C="tests/test_gpu_cull.py tests/test_gpu_prm.py tests/test_gpu_fullsize.py::test_cfg4_chain_culled_scan_1e6 tests/test_gpu_fullsize.py::test_cfg4_every_milestone_vs_exact_scan"
timeout -k 10 400 python -u -m pytest $TESTS_C -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest_q16.log" 2>&1
rc=$?; echo "chain q16: $(tail -1 "$out/pytest_q16.log")"; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh cfg4 "--workload cfg4" 2 - OMPL_GPU_CHAIN_Q16=0 || exit 1
TESTS_K="tests/test_gpu_nn.py tests/test_gpu_fullsize.py::test_cfg3_every_query_vs_exact_scan tests/test_gpu_fullsize.py::test_cfg5k_every_vertex_vs_exact_scan"
OMPL_GPU_KNN_Q16=1 timeout -k 10 400 python -u -m pytest $TESTS_K -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/pytest_kq16.log" 2>&1
rc=$?; echo "knn q16: $(tail -1 "$out/pytest_kq16.log")"; rc_ok $rc "knn q16"
bash tools/ab_env.sh cfg5k "--workload cfg5 --bitstar-knn" 2 - OMPL_GPU_KNN_Q16=1 || exit 1
bash tools/ab_env.sh cfg3q "--workload cfg3" 1 - OMPL_GPU_KNN_Q16=1 || exit 1
TESTS_Q="tests/test_gpu_batch.py tests/test_gpu_bitstar.py tests/test_gpu_fullsize.py::test_cfg5_every_vertex_radius_vs_exact_scan tests/test_gpu_fullsize.py::test_cfg5_radius_1e7_valid_samples"
OMPL_GPU_RADIUS_Q16=1 timeout -k 10 400 python -u -m pytest $TESTS_Q -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/pytest_rq16.log" 2>&1
rc=$?; echo "radius q16: $(tail -1 "$out/pytest_rq16.log")"; rc_ok $rc "radius q16"
bash tools/ab_env.sh cfg5 "--workload cfg5" 2 - OMPL_GPU_RADIUS_Q16=1 || exit 1
fi
if [ "$P" = 3 ]; then  # the radius walk's occupancy / per-query-mask variants
TESTS_R="tests/test_gpu_fullsize.py::test_cfg5_every_vertex_radius_vs_exact_scan tests/test_gpu_fullsize.py::test_cfg5_radius_1e7_valid_samples"
for v in 11 13; do
  OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var$v.so timeout -k 10 300 python -u -m pytest $TESTS_R -m gpu -x -q --timeout 200 \
      --timeout-method thread > "$out/pytest_r$v.log" 2>&1
  rc=$?; echo "var$v radius: $(tail -1 "$out/pytest_r$v.log")"; rc_ok $rc var$v
done
bash tools/ab_env.sh cfg5v "--workload cfg5" 1 - VAR=5 VAR=6 VAR=11 VAR=13 || exit 1
fi
if [ "$P" = 5 ]; then  # the chain cull with the next tile in flight; radius 16-bit default
T5="tests/test_gpu_prm.py tests/test_gpu_fullsize.py::test_cfg4_every_milestone_vs_exact_scan"
OMPL_GPU_CHAIN_PREFETCH=1 timeout -k 10 400 python -u -m pytest $T5 -m gpu -x -q --timeout 300 --timeout-method thread \
    > "$out/pytest_pf.log" 2>&1
rc=$?; echo "chain prefetch: $(tail -1 "$out/pytest_pf.log")"; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh cfg4pf "--workload cfg4" 2 - OMPL_GPU_CHAIN_PREFETCH=1 || exit 1
fi
if [ "$P" = 6 ]; then  # chunks of the chain cull's MODE 2 pass (waves per CU) now that thresholds are shared
bash tools/ab_env.sh cfg4wpc "--workload cfg4" 1 - OMPL_GPU_CHAIN_WPC=24 OMPL_GPU_CHAIN_WPC=48 OMPL_GPU_CHAIN_WPC=192 OMPL_GPU_CHAIN_WPC=384 || exit 1
fi
if [ "$P" = 7 ]; then  # the chunk cap of the chain cull's MODE 2 pass
bash tools/ab_env.sh cfg4s "--workload cfg4" 1 - "OMPL_GPU_CHAIN_WPC=1024 OMPL_GPU_CHAIN_SMAX=128" "OMPL_GPU_CHAIN_WPC=1024 OMPL_GPU_CHAIN_SMAX=256" - || exit 1
timeout -k 10 300 python -u -m pytest tests/test_gpu_prm.py tests/test_gpu_fullsize.py::test_cfg4_every_milestone_vs_exact_scan -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_wpc.log" 2>&1
rc=$?; echo "wpc 384: $(tail -1 "$out/pytest_wpc.log")"; [ $rc = 0 ] || exit 1
fi
if [ "$P" = 8 ]; then  # chain chunks: blocks nearest the home tile first
OMPL_GPU_CHAIN_KDORDER=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_prm.py tests/test_gpu_cull.py tests/test_gpu_fullsize.py::test_cfg4_every_milestone_vs_exact_scan -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_kdo.log" 2>&1
rc=$?; echo "kd order: $(tail -1 "$out/pytest_kdo.log")"; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh cfg4kdo "--workload cfg4" 2 - OMPL_GPU_CHAIN_KDORDER=1 || exit 1
fi
if [ "$P" = 9 ]; then  # queries per wave of the 64-lane (k = 57) group walk
for v in 14 15; do
  OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py::test_cfg5k_every_vertex_vs_exact_scan tests/test_gpu_nn.py -m gpu -x -q --timeout 200 \
      --timeout-method thread > "$out/pytest_g$v.log" 2>&1
  rc=$?; echo "var$v: $(tail -1 "$out/pytest_g$v.log")"; rc_ok $rc var$v
done
bash tools/ab_env.sh cfg5kg "--workload cfg5 --bitstar-knn" 2 - VAR=14 VAR=15 || exit 1
fi
if [ "$P" = 10 ]; then  # the chain pre-pass in parts (atomicMin of the parts' K2-th keys)
OMPL_GPU_CHAIN_TAU_PARTS=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_prm.py tests/test_gpu_cull.py tests/test_gpu_fullsize.py::test_cfg4_every_milestone_vs_exact_scan -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_tp.log" 2>&1
rc=$?; echo "tau parts: $(tail -1 "$out/pytest_tp.log")"; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh cfg4tp "--workload cfg4" 2 - OMPL_GPU_CHAIN_TAU_PARTS=2 OMPL_GPU_CHAIN_TAU_PARTS=4 || exit 1
fi
if [ "$P" = 11 ]; then  # queries per wave: SE3 G = 2 on cfg3 (variant 15), R^n G = 4 on cfg2 (variant 16)
for v in 15 16; do
  OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py tests/test_gpu_cull.py -m gpu -x -q --timeout 200 \
      --timeout-method thread > "$out/pytest_g$v.log" 2>&1
  rc=$?; echo "var$v: $(tail -1 "$out/pytest_g$v.log")"; rc_ok $rc var$v
done
bash tools/ab_env.sh cfg3g "--workload cfg3" 2 - VAR=15 || exit 1
bash tools/ab_env.sh cfg2g "--workload cfg2" 2 - VAR=16 || exit 1
fi
if [ "$P" = 12 ]; then  # chain lists of sorted positions (AoS certificate rows)
timeout -k 10 400 python -u -m pytest tests/test_gpu_prm.py tests/test_gpu_cull.py tests/test_gpu_nn.py tests/test_gpu_fullsize.py::test_cfg4_every_milestone_vs_exact_scan tests/test_gpu_fullsize.py::test_cfg4_chain_culled_scan_1e6 -m gpu -x -q --timeout 300 --timeout-method thread > "$out/pytest_pos.log" 2>&1
rc=$?; echo "chain positions: $(tail -1 "$out/pytest_pos.log")"; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh cfg4pos "--workload cfg4" 2 - || exit 1
bash tools/prof_workload.sh cfg4 r4_cfg4 || exit 1
fi
if [ "$P" = 13 ]; then  # R^n G = 2 (variant 17, cfg2); radius slab walk G = 2 (variant 18, cfg5)
OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var17.so timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py tests/test_gpu_cull.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_g17.log" 2>&1
rc=$?; echo "var17: $(tail -1 "$out/pytest_g17.log")"; rc_ok $rc var17
OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var18.so timeout -k 10 300 python -u -m pytest tests/test_gpu_fullsize.py::test_cfg5_every_vertex_radius_vs_exact_scan tests/test_gpu_fullsize.py::test_cfg5_radius_1e7_valid_samples tests/test_gpu_batch.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_g18.log" 2>&1
rc=$?; echo "var18: $(tail -1 "$out/pytest_g18.log")"; rc_ok $rc var18
bash tools/ab_env.sh cfg2g2 "--workload cfg2" 2 - VAR=17 || exit 1
bash tools/ab_env.sh cfg5g2 "--workload cfg5" 2 - VAR=18 || exit 1
bash tools/ab_env.sh cfg3g2 "--workload cfg3" 1 - || exit 1
fi
if [ "$P" = 14 ]; then  # the SE3 walk held to 64 VGPRs (8 waves per SIMD, variant 19) on cfg3 and cfg5k; R^n G = 2 product on cfg2
OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var19.so timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py tests/test_gpu_cull.py -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_g19.log" 2>&1
rc=$?; echo "var19: $(tail -1 "$out/pytest_g19.log")"; rc_ok $rc var19
timeout -k 10 300 python -u -m pytest tests/test_gpu_nn.py tests/test_gpu_cull.py tests/test_gpu_fullsize.py::test_cfg2_every_query_vs_exact_scan tests/test_gpu_fullsize.py::test_cfg2_reference_store_k10 -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_rv2.log" 2>&1
rc=$?; echo "rv G=2: $(tail -1 "$out/pytest_rv2.log")"; [ $rc = 0 ] || exit 1
bash tools/ab_env.sh cfg3w8 "--workload cfg3" 2 - VAR=19 || exit 1
bash tools/ab_env.sh cfg5kw8 "--workload cfg5 --bitstar-knn" 1 - VAR=19 || exit 1
bash tools/ab_env.sh cfg2p "--workload cfg2" 1 - || exit 1
fi
if [ "$P" = 15 ]; then  # the bulk-merge threshold of the group walk at G = 2
bash tools/ab_env.sh cfg3bulk "--workload cfg3" 2 - OMPL_GPU_BULK=4 OMPL_GPU_BULK=16 || exit 1
bash tools/ab_env.sh cfg5kbulk "--workload cfg5 --bitstar-knn" 1 - OMPL_GPU_BULK=4 OMPL_GPU_BULK=16 || exit 1
bash tools/ab_env.sh cfg2bulk "--workload cfg2" 1 - OMPL_GPU_BULK=4 OMPL_GPU_BULK=16 || exit 1
fi
if [ "$P" = 16 ]; then  # the bulk-merge threshold, wider
bash tools/ab_env.sh cfg3bulk2 "--workload cfg3" 2 OMPL_GPU_BULK=16 OMPL_GPU_BULK=32 OMPL_GPU_BULK=64 || exit 1
bash tools/ab_env.sh cfg5kbulk2 "--workload cfg5 --bitstar-knn" 1 OMPL_GPU_BULK=16 OMPL_GPU_BULK=32 OMPL_GPU_BULK=64 || exit 1
fi
if [ "$P" = 17 ]; then  # chain cull at 4 queries per wave (variant 20); the super-tile re-check at G = 2
OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var20.so timeout -k 10 300 python -u -m pytest tests/test_gpu_prm.py tests/test_gpu_cull.py tests/test_gpu_fullsize.py::test_cfg4_every_milestone_vs_exact_scan -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_g20.log" 2>&1
rc=$?; echo "var20: $(tail -1 "$out/pytest_g20.log")"; rc_ok $rc var20
bash tools/ab_env.sh cfg4g4 "--workload cfg4" 2 - VAR=20 || exit 1
bash tools/ab_env.sh cfg3rc "--workload cfg3" 2 - OMPL_GPU_SUPER_RECHECK=0 || exit 1
fi
if [ "$P" = 18 ]; then  # chain cull at 2 queries per wave (variant 21)
OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var21.so timeout -k 10 300 python -u -m pytest tests/test_gpu_prm.py tests/test_gpu_cull.py tests/test_gpu_fullsize.py::test_cfg4_every_milestone_vs_exact_scan -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_g21.log" 2>&1
rc=$?; echo "var21: $(tail -1 "$out/pytest_g21.log")"; rc_ok $rc var21
bash tools/ab_env.sh cfg4g2 "--workload cfg4" 2 - VAR=21 || exit 1
fi
if [ "$P" = 19 ]; then  # the popped super-tile re-check at G = 2, more reps
bash tools/ab_env.sh cfg3rc2 "--workload cfg3" 3 - OMPL_GPU_SUPER_RECHECK=0 || exit 1
bash tools/ab_env.sh cfg5krc "--workload cfg5 --bitstar-knn" 2 - OMPL_GPU_SUPER_RECHECK=0 || exit 1
fi
if [ "$P" = 20 ]; then  # the chain pre-pass window: 32 / 8 tiles (variants 22 / 23)
for v in 22 23; do
  OMPL_GPU_LIB=tools/probe_lib/libompl_gpu_var$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_prm.py tests/test_gpu_fullsize.py::test_cfg4_every_milestone_vs_exact_scan -m gpu -x -q --timeout 200 --timeout-method thread > "$out/pytest_t$v.log" 2>&1
  rc=$?; echo "var$v: $(tail -1 "$out/pytest_t$v.log")"; rc_ok $rc var$v
done
bash tools/ab_env.sh cfg4tw "--workload cfg4" 2 - VAR=22 VAR=23 || exit 1
fi
