#!/bin/bash
# The round-6 GPU sessions, one case per run tag (outputs: gpurun_out/<tag>/, copied to
# profiles/r06/<tag>/ when DESIGN.md cites them). usage (via gpurun): bash tools/gpu_r06_runs.sh <tag>
# Cases r06d-r06h ran the treelet wavefront, since archived (profiles/archive/experiments/); they
# need that code applied again. Cases naming abship/ libraries need those A/B builds
# (tools/build_at_commit.py, tools/build_variant.py) in abship/ first.
set -o pipefail
T=$1
mkdir -p gpurun_out/$T
case "$T" in
  r06a)
    # C2 regression bisect: the round-4 final kernel and each round-5 kernel commit against the
    # round-5 head, one process (tools/build_at_commit.py builds, abvar/bisect/)
    L="abvar/bisect/lib_797545e.so"
    for c in fcb6cf7 3e2677f f524fdb 25c7b12 a054092 6da6bce 37b2ecf; do L="$L abvar/bisect/lib_$c.so"; done
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    ;;
  r06b)
    # the cleaned ABI-12 build: every GPU test, smoke, then same-process A/B against the r05
    # head and the r04 final builds on C2, C3, C5
    timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || exit 1
    L="rust_gpu_raytracing_amd/librt_pathtrace.so abvar/bisect/lib_797545e.so abvar/bisect/lib_fcb6cf7.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 5 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c5.json 2> gpurun_out/$T/ab_c5.err || exit 1
    timeout -k 10 300 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/$T/brute_tiled.json 2> gpurun_out/$T/brute_tiled.err || exit 1
    timeout -k 10 300 python3 bench.py --config c5_heightfield --brute-force stream --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/$T/brute_stream.json 2> gpurun_out/$T/brute_stream.err || exit 1
    timeout -k 10 300 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit 1
    ;;
  r06c)
    # what the C2 kernel time is sensitive to: the culling bound's range check compiled out
    # (diagnostic), loop alignment off, non-fallthrough blocks aligned to 64 B
    L="rust_gpu_raytracing_amd/librt_pathtrace.so abvar/bisect/lib_fcb6cf7.so abvar/r06c/lib_noguard.so abvar/r06c/lib_noalign.so abvar/r06c/lib_blk64.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 5 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c5.json 2> gpurun_out/$T/ab_c5.err || exit 1
    # the bench step's wall time against its launch span (one 20-frame launch between syncs)
    timeout -k 10 200 python3 tools/launch_gap.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/bisect/lib_797545e.so abvar/bisect/lib_fcb6cf7.so > gpurun_out/$T/launch_gap.jsonl 2> gpurun_out/$T/launch_gap.err || exit 1
    timeout -k 10 200 python3 bench.py --no-cpu-baseline > gpurun_out/$T/bench1.json 2> gpurun_out/$T/bench1.err || exit 1
    timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-cadences > gpurun_out/$T/bench2.json 2> gpurun_out/$T/bench2.err || exit 1
    ;;
  r06d)
    # the treelet wavefront: its GPU tests, then C5 against the persistent walk (same process and bench)
    timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -m gpu -k "treelet or environment or tuning" > gpurun_out/$T/tests.log 2>&1 || exit 1
    timeout -k 10 400 python3 tools/ab_env.py "" "treelet_walk=1" --config c5_heightfield --frame-batch 20 --frames 40 --rounds 3 > gpurun_out/$T/ab_c5.jsonl 2> gpurun_out/$T/ab_c5.err || exit 1
    timeout -k 10 300 python3 bench.py --config c5_heightfield --tune treelet_walk=1 --no-cpu-baseline --no-cadences > gpurun_out/$T/bench_c5_tl.json 2> gpurun_out/$T/bench_c5_tl.err || exit 1
    timeout -k 10 300 python3 bench.py --config c5_heightfield --no-cpu-baseline --no-cadences > gpurun_out/$T/bench_c5.json 2> gpurun_out/$T/bench_c5.err || exit 1
    ;;
  r06e)
    # where the treelet wavefront's time goes on C5: kernel trace of the bench (per-kernel stats;
    # the count of rt_tl_top_kernel launches is the number of rounds)
    export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/trace -o run -- python3 bench.py --config c5_heightfield --tune treelet_walk=1 --steps 20 --warmup 20 --settle-ms 0 --no-cpu-baseline --no-cadences > gpurun_out/$T/trace_bench.json 2> gpurun_out/$T/trace.err || exit 1
    ;;
  r06f)
    # the treelet wavefront's kernels under SQ counters (one 4-frame C5 batch per pass)
    export TMPDIR=/tmp
    B="bench.py --config c5_heightfield --tune treelet_walk=1 --steps 4 --warmup 0 --settle-ms 0 --no-cpu-baseline --no-cadences"
    timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/$T/pmc_a -o run -- python3 $B > gpurun_out/$T/a.json 2> gpurun_out/$T/a.err || exit 1
    timeout -s KILL 120 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/$T/pmc_b -o run -- python3 $B > gpurun_out/$T/b.json 2> gpurun_out/$T/b.err || exit 1
    ;;
  r06g)
    # first hardware pass of the ABI-12 build and the treelet wavefront: every GPU test, smoke,
    # the headline bench, C5 persistent walk vs treelet wavefront, both brute-force lines
    timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || exit 1
    timeout -k 10 300 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit 1
    timeout -k 10 300 python3 tools/ab_env.py "" "treelet_walk=1" --config c5_heightfield --frame-batch 20 --frames 40 --rounds 3 > gpurun_out/$T/ab_c5.jsonl 2> gpurun_out/$T/ab_c5.err || exit 1
    timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/$T/brute_tiled.json 2> gpurun_out/$T/brute_tiled.err || exit 1
    timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force stream --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/$T/brute_stream.json 2> gpurun_out/$T/brute_stream.err || exit 1
    ;;
  r06h)
    # the ABI-12 head against the round-4 final (fcb6cf7) and round-5 head (797545e) kernels in one
    # process (abship/, tools/build_at_commit.py), then the treelet wavefront's kernel trace on C5
    L="rust_gpu_raytracing_amd/librt_pathtrace.so abship/lib_fcb6cf7.so abship/lib_797545e.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 5 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c5.json 2> gpurun_out/$T/ab_c5.err || exit 1
    export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$T/trace -o run -- python3 bench.py --config c5_heightfield --tune treelet_walk=1 --steps 20 --warmup 20 --settle-ms 0 --no-cpu-baseline --no-cadences > gpurun_out/$T/trace_bench.json 2> gpurun_out/$T/trace.err || exit 1
    ;;
  r06i)
    # the culling bound's range check as a bit-mask merge (no branch) against the round-4 final
    # and round-5 head kernels, C2/C3/C5 in one process
    L="rust_gpu_raytracing_amd/librt_pathtrace.so abship/lib_fcb6cf7.so abship/lib_797545e.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 5 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cadences > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit 1
    ;;
  r06j)
    # the build without the treelet wavefront: every GPU test, smoke, the headline bench; then
    # the RT_DIAG split of C2 and C3 (where the idle lanes are)
    timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || exit 1
    timeout -k 10 300 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit 1
    RT_LIB=abship/lib_diag.so timeout -k 10 300 python3 tools/diag_split.py --frame-batch 20 c2_rtiow c3_chess > gpurun_out/$T/diag_split.jsonl 2> gpurun_out/$T/diag_split.err || exit 1
    ;;
  r06k)
    # sphere-only walks: the group tests of a block of unrolled node steps run once for every lane
    # that reached a leaf in it (the product build, 3 steps), against the previous build (head) and
    # blocks of 2/4/6 steps; every GPU test first
    timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    L="rust_gpu_raytracing_amd/librt_pathtrace.so abship/lib_head.so abship/lib_blk2.so abship/lib_blk4.so abship/lib_blk6.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c1_four_spheres --width 800 --height 600 --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c1.json 2> gpurun_out/$T/ab_c1.err || exit 1
    timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-cadences > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit 1
    ;;
  r06l)
    # block sizes of the sphere-only group tests: 4, 5, 6, 8, 12 unrolled node steps
    L="abship/lib_blk4.so abship/lib_blk5.so abship/lib_blk6.so abship/lib_blk8.so abship/lib_blk12.so abship/lib_head.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c1_four_spheres --width 800 --height 600 --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c1.json 2> gpurun_out/$T/ab_c1.err || exit 1
    RT_LIB=abship/lib_diag.so timeout -k 10 300 python3 tools/diag_split.py --frame-batch 20 c2_rtiow > gpurun_out/$T/diag_split.jsonl 2> gpurun_out/$T/diag_split.err || exit 1
    ;;
  r06m)
    # the sphere-only block group tests: lanes waiting at their leaf (blk) or walking on past it
    # until a second leaf (wo), blocks of 4 and 6 node steps
    L="abship/lib_blk4.so abship/lib_blk6.so abship/lib_wo4.so abship/lib_wo6.so abship/lib_head.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 11 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    ;;
  r06n)
    # the sphere group test's candidate arms as a per-lane loop over its candidates (cand) against
    # the four predicated arms (b6, the product build): C2, C4
    L="abship/lib_b6.so abship/lib_cand.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 11 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    ;;
  r06o)
    # adaptive block group tests: after every block of U node steps, once W/8 of the traversing
    # lanes wait at a leaf (ad<U>_<W>), against the fixed 6-step block (b6, the product build)
    L="abship/lib_b6.so abship/lib_ad3_2.so abship/lib_ad3_4.so abship/lib_ad2_3.so abship/lib_ad4_3.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 11 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    ;;
  r06p)
    # adaptive block group tests around blocks of 4 steps and a 3/8 waiting share
    L="abship/lib_ad4_3.so abship/lib_ad4_2.so abship/lib_ad4_4.so abship/lib_ad5_3.so abship/lib_ad6_3.so abship/lib_ad3_3.so abship/lib_ad4_5.so abship/lib_b6.so"
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 11 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py abship/lib_ad4_3.so abship/lib_b6.so abship/lib_head.so --config c1_four_spheres --width 800 --height 600 --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c1.json 2> gpurun_out/$T/ab_c1.err || exit 1
    ;;
  r06q)
    # the adaptive block build: every GPU test, smoke, A/B against the round's first build (head)
    # on C1-C4, the headline bench, and the RT_DIAG split of C2
    timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || exit 1
    L="rust_gpu_raytracing_amd/librt_pathtrace.so abship/lib_head.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 5 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 300 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit 1
    RT_LIB=abship/lib_diag.so timeout -k 10 300 python3 tools/diag_split.py --frame-batch 20 c2_rtiow > gpurun_out/$T/diag_split.jsonl 2> gpurun_out/$T/diag_split.err || exit 1
    ;;
  r06r)
    # mode-2 (LDS-resident triangle walk) leaf batches fused into the node-step iteration (fuse2),
    # at batch shares 6/8 (the scene default), 4/8, 3/8, 2/8, against the product build
    L="abship/lib_final.so abship/lib_fuse2.so abship/lib_fuse2.so:leaf_batch=4 abship/lib_fuse2.so:leaf_batch=3 abship/lib_fuse2.so:leaf_batch=2"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    ;;
  r06s)
    # fused mode-2 leaf batches: shares 6/7/8 eighths, node-step blocks of 1, 2 (fuse2), 3
    L="abship/lib_fuse2.so abship/lib_fuse2.so:leaf_batch=7 abship/lib_fuse2.so:leaf_batch=8 abship/lib_fuse2u3.so abship/lib_fuse2u3.so:leaf_batch=7 abship/lib_fuse2u1.so abship/lib_fuse2u1.so:leaf_batch=7"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 500 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    ;;
  r06t)
    # fused mode-2 leaf batches: node-step blocks of 3, 4, 5 at shares 5/8 and 6/8
    L="abship/lib_fuse2u3.so abship/lib_fuse2u3.so:leaf_batch=5 abship/lib_fuse2u4.so abship/lib_fuse2u4.so:leaf_batch=5 abship/lib_fuse2u5.so abship/lib_fuse2u5.so:leaf_batch=5 abship/lib_final.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 500 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    ;;
  r06u)
    # the fused mode-2 leaf batch build (f2, the product): every GPU test; then the cooperative
    # batches of the global-memory walks fused the same way (f1) on C5, against f2
    timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    L="abship/lib_f2.so abship/lib_f1.so abship/lib_f1.so:leaf_batch=5 abship/lib_f1.so:leaf_batch=3"
    timeout -k 10 500 python3 tools/ab_bench.py $L --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c5.json 2> gpurun_out/$T/ab_c5.err || exit 1
    ;;
  r06v)
    # traversal thresholds at the new build (the wave goes back to shading once this many lanes
    # still traverse): C2 (default 8) 4/12/16, C3 (default 24) 16/32
    F=abship/lib_f2.so
    timeout -k 10 300 python3 tools/ab_bench.py $F $F:trav_threshold=4 $F:trav_threshold=12 $F:trav_threshold=16 --config c2_rtiow --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $F $F:trav_threshold=16 $F:trav_threshold=32 --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    ;;
  r06w)
    # traversal thresholds, second pass: C2 10/12/14/20, C3 and C4 28/32/40
    F=abship/lib_f2.so
    timeout -k 10 300 python3 tools/ab_bench.py $F $F:trav_threshold=10 $F:trav_threshold=12 $F:trav_threshold=14 $F:trav_threshold=20 --config c2_rtiow --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $F $F:trav_threshold=28 $F:trav_threshold=32 $F:trav_threshold=40 --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py $F $F:trav_threshold=28 $F:trav_threshold=32 $F:trav_threshold=40 --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    ;;
  r06x1)
    # final-build profiles (kernel trace + FETCH/WRITE/SQ passes, tools/profile.sh): C2, C3, C4 (3840x2160)
    timeout -k 10 600 bash tools/profile.sh r06_c2 > gpurun_out/$T.c2.log 2>&1 || exit 1
    timeout -k 10 600 bash tools/profile.sh r06_c3 --config c3_chess > gpurun_out/$T.c3.log 2>&1 || exit 1
    timeout -k 10 600 bash tools/profile.sh r06_c4k --config c4_mixed --width 3840 --height 2160 > gpurun_out/$T.c4k.log 2>&1 || exit 1
    ;;
  r06x2)
    # final-build profiles: C5 (exact walk), C5 brute force (LDS tiles, scalar-cache stream)
    timeout -k 10 600 bash tools/profile.sh r06_c5 --config c5_heightfield > gpurun_out/$T.c5.log 2>&1 || exit 1
    timeout -k 10 600 bash tools/profile.sh r06_c5b --config c5_heightfield --brute-force --steps 2 --warmup 2 > gpurun_out/$T.c5b.log 2>&1 || exit 1
    timeout -k 10 600 bash tools/profile.sh r06_c5bs --config c5_heightfield --brute-force stream --steps 2 --warmup 2 > gpurun_out/$T.c5bs.log 2>&1 || exit 1
    ;;
  r06x3)
    # final-build profile of C4 at its BASELINE size (3840x2160, 16 bounces)
    timeout -k 10 600 bash tools/profile.sh r06_c4k --config c4_mixed --width 3840 --height 2160 > gpurun_out/$T.c4k.log 2>&1 || exit 1
    # and the C5 walk's L1/TA/TD counters at the final build (tools/pmc_tcp.sh)
    timeout -k 10 600 bash tools/pmc_tcp.sh r06_c5tcp --config c5_heightfield > gpurun_out/$T.c5tcp.log 2>&1 || exit 1
    ;;
  r06y2)
    # the new leaf-scheduling test; then, in triangle kernels, sphere-phase lanes waiting at their
    # leaf (sphwait) instead of walking on, on C4
    timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k leaf_scheduling > gpurun_out/$T/tests.log 2>&1 || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py abship/lib_f3.so abship/lib_sphwait.so --config c4_mixed --width 3840 --height 2160 --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    ;;
  r06y3)
    # the decoupled drain for every instance (dd): C2's N=1 and N=8 shares, predicted by the probe,
    # at drain thresholds / minimum steps, against the product build
    P="python3 tools/strong_probe.py --steps 20 --gather accumulation --ns 1 8 --repeats 3"
    timeout -k 10 200 $P > gpurun_out/$T/prod.jsonl 2> gpurun_out/$T/prod.err || exit 1
    RT_LIB=abship/lib_dd.so timeout -k 10 200 $P > gpurun_out/$T/dd.jsonl 2> gpurun_out/$T/dd.err || exit 1
    RT_LIB=abship/lib_dd.so timeout -k 10 200 $P --tune drain_threshold=16 > gpurun_out/$T/dd_t16.jsonl 2> gpurun_out/$T/dd_t16.err || exit 1
    RT_LIB=abship/lib_dd.so timeout -k 10 200 $P --tune drain_threshold=48 drain_min_steps=16 > gpurun_out/$T/dd_t48m16.jsonl 2> gpurun_out/$T/dd_t48m16.err || exit 1
    RT_LIB=abship/lib_dd.so timeout -k 10 200 $P --tune drain_min_steps=8 > gpurun_out/$T/dd_m8.jsonl 2> gpurun_out/$T/dd_m8.err || exit 1
    ;;
  r06y4)
    # the packet pre-pass reading its records with scalar loads (the product build now) against
    # the final profiled build (f3): every GPU test, then C5 in one process (wall and spans)
    timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    timeout -k 10 500 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abship/lib_f3.so --config c5_heightfield --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c5.json 2> gpurun_out/$T/ab_c5.err || exit 1
    timeout -k 10 300 python3 bench.py --config c5_heightfield --no-cpu-baseline --no-cadences > gpurun_out/$T/bench_c5.json 2> gpurun_out/$T/bench_c5.err || exit 1
    ;;
  r06y5)
    # the sphere group test's candidate arms as selects instead of branches (csel)
    L="abship/lib_f3.so abship/lib_csel.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 11 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    ;;
  r06y6)
    # the RT_DIAG split at the final build: C2, C3, C4 (1920x1080)
    RT_LIB=abship/lib_diag.so timeout -k 10 300 python3 tools/diag_split.py --frame-batch 20 c2_rtiow c3_chess c4_mixed > gpurun_out/$T/diag_split.jsonl 2> gpurun_out/$T/diag_split.err || exit 1
    ;;
  r06y7)
    # triangle walks that end wait for one phase switch per block (pd) instead of switching to the
    # sphere walk inside every node step: the parity tests on that build, then C3/C4/C5 A/B
    RT_LIB=abship/lib_pd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    L="abship/lib_f3.so abship/lib_pd.so"
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c5.json 2> gpurun_out/$T/ab_c5.err || exit 1
    ;;
  r06y8)
    # a tile's frames claimed from one stripe, i.e. on one XCD (xcd), against the product build (f3):
    # the frame-batch parity tests on that build, then C5, C4, C3, C2 in one process
    RT_LIB=abship/lib_xcd.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "frame_batch or full_frame_baseline_size or sampled_c5 or leaf_scheduling or cost_ordered or tile_split or overlapped" > gpurun_out/$T/tests.log 2>&1 || exit 1
    L="abship/lib_f3.so abship/lib_xcd.so"
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c5_heightfield --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c5.json 2> gpurun_out/$T/ab_c5.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    ;;
  r06y9)
    # mode-2 leaf batches of one kind (the triangle or the sphere leaves, whichever more lanes hold)
    # instead of both (ps): the leaf tests on that build, then C4 and C3
    RT_LIB=abship/lib_ps.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "leaf_scheduling or fuzz or c4 or mixed" > gpurun_out/$T/tests.log 2>&1 || exit 1
    L="abship/lib_f3.so abship/lib_ps.so"
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    ;;
  r06v1)
    # single-kind mode-2 leaf batches (the product build, f4): every GPU test, smoke, A/B against
    # the previous final build (f3) on C2, C3, C4
    timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || exit 1
    L="abship/lib_f3.so abship/lib_f4.so"
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    ;;
  r06v2)
    # the product build (f5: single-kind leaf batches, two ballots): every GPU test, smoke, A/B
    # against f3 on C4/C3/C2, then the final-build profiles of C2, C3, C4 (r06x1)
    timeout -k 10 600 python3 -u -m pytest tests/ -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || exit 1
    L="abship/lib_f3.so abship/lib_f5.so"
    timeout -k 10 400 python3 tools/ab_bench.py $L --config c4_mixed --width 3840 --height 2160 --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $L --config c2_rtiow --rounds 9 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c2.json 2> gpurun_out/$T/ab_c2.err || exit 1
    bash tools/gpu_r06_runs.sh r06x1 || exit 1
    ;;
  r06v3)
    # knob re-check at the final build (runtime tuning, no rebuild): C4 and C3 leaf-batch shares
    # and traversal thresholds
    F=abship/lib_f5.so
    timeout -k 10 500 python3 tools/ab_bench.py $F $F:leaf_batch=5 $F:leaf_batch=7 $F:trav_threshold=16 $F:trav_threshold=32 --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/$T/ab_c4.json 2> gpurun_out/$T/ab_c4.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py $F $F:leaf_batch=5 $F:leaf_batch=7 $F:trav_threshold=16 $F:trav_threshold=32 --config c3_chess --rounds 7 --frames 60 --frame-batch 20 > gpurun_out/$T/ab_c3.json 2> gpurun_out/$T/ab_c3.err || exit 1
    ;;
  r06z)
    # the final pass: every GPU test, smoke, the headline bench, the library rebuilt from source on
    # the box and its parity tests (provenance: DESIGN.md §6), all configurations, strong probe
    timeout -k 10 900 python3 -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/$T/tests.log 2>&1 || exit 1
    timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$T/smoke.log 2>&1 || exit 1
    timeout -k 10 300 python3 bench.py > gpurun_out/$T/bench.json 2> gpurun_out/$T/bench.err || exit 1
    timeout -k 10 600 python3 -c "
import subprocess, pathlib
from rust_gpu_raytracing_amd import build as b
subprocess.run(b.hipcc_command(pathlib.Path('/tmp/librt_srcbuild.so')), check=True)
print('built /tmp/librt_srcbuild.so, sources', b.source_hash())" > gpurun_out/$T/srcbuild.log 2>&1 || exit 1
    RT_LIB=/tmp/librt_srcbuild.so timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "golden or full_frame_baseline_size" >> gpurun_out/$T/srcbuild.log 2>&1 || exit 1
    RT_LIB=/tmp/librt_srcbuild.so timeout -k 10 100 python3 -c "
from rust_gpu_raytracing_amd import _native as N, build as b
lib = N.load_library()
print('srcbuild library hash', lib.rt_build_hash().decode(), '== tree', b.source_hash())" >> gpurun_out/$T/srcbuild.log 2>&1 || exit 1
    timeout -k 10 600 python3 tools/bench_all.py --frames 20 > gpurun_out/$T/bench_all.jsonl 2> gpurun_out/$T/bench_all.err || exit 1
    ;;
  r06z2)
    # strong-scaling probes at the final build, the bench's accumulation payload: C2, C4
    timeout -k 10 400 python3 tools/strong_probe.py --steps 20 --gather accumulation > gpurun_out/$T/strong_c2_accumulation.jsonl 2> gpurun_out/$T/strong_c2.err || exit 1
    timeout -k 10 500 python3 tools/strong_probe.py --config c4_mixed --steps 20 --gather accumulation > gpurun_out/$T/strong_c4_accumulation.jsonl 2> gpurun_out/$T/strong_c4.err || exit 1
    ;;
  *)
    echo "unknown tag $T"; exit 2
    ;;
esac
