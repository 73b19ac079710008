#!/bin/bash
# The round-5 GPU sessions, one case per run tag (their outputs: gpurun_out/<tag>/, the files
# DESIGN.md and profiles/r05 cite). usage (via gpurun): bash tools/gpu_r05_runs.sh <tag>
# Some cases load experiment builds (abvar/*.so, tools/build_variant.py with the -D switch
# named in the comment) or need the source state of the run (see the git log of that day).
set -o pipefail
case "$1" in
  r05h)
    # walk-variant and brute-force tests, q4 A/B, brute A/B
    mkdir -p gpurun_out/r05h
    timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "global_walk_variants or lds_vertex or brute" > gpurun_out/r05h/tests.log 2>&1 || exit 1
    RT_BRUTE_WF=1 timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05h/brute_wf.json 2> gpurun_out/r05h/brute_wf.err || exit 1
    RT_BRUTE_WF=0 timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05h/brute_old.json 2> gpurun_out/r05h/brute_old.err || exit 1
    timeout -k 10 400 python3 tools/ab_env.py "RT_TRI_Q4=1" "RT_TRI_Q4=0" "RT_TRI_Q4=1 RT_BLOCK_THREADS=512" "RT_TRI_Q4=1 RT_BLOCK_THREADS=256" --config c5_heightfield --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05h/ab_threads.jsonl 2> gpurun_out/r05h/ab_threads.err || exit 1
    RT_LIB=abvar/lib_diag.so RT_TRI_Q4=1 timeout -k 10 200 python3 tools/diag_split.py --frame-batch 20 c5_heightfield > gpurun_out/r05h/diag_q4.json 2>&1 || exit 1
    RT_LIB=abvar/lib_diag.so RT_TRI_Q4=0 timeout -k 10 200 python3 tools/diag_split.py --frame-batch 20 c5_heightfield > gpurun_out/r05h/diag_bin.json 2>&1
    ;;
  r05i)
    # brute-force tests + bench, C5 layout A/B
    mkdir -p gpurun_out/r05i
    timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "brute" > gpurun_out/r05i/tests.log 2>&1 || exit 1
    timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05i/brute_wf.json 2> gpurun_out/r05i/brute_wf.err || exit 1
    timeout -k 10 400 python3 tools/ab_env.py "RT_TRI_OCTANTS=1" "RT_TRI_OCTANTS=0" "RT_TRI_OCTANTS=0 RT_TRI_QNODES=0" "RT_TRI_OCTANTS=1 RT_PRIMARY_PASS=0" "RT_TRI_OCTANTS=0 RT_PRIMARY_PASS=0" --config c5_heightfield --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05i/ab_oct.jsonl 2> gpurun_out/r05i/ab_oct.err
    ;;
  r05j)
    # PMC of the C5 walk (TCP/TA/TD) and of the brute-force wavefront
    bash tools/pmc_tcp.sh r05_c5tcp --config c5_heightfield || exit 1
    bash tools/profile.sh r05_c5b --config c5_heightfield --brute-force --steps 2 --warmup 2 || exit 1
    ;;
  r05k)
    # brute-force wavefront variants
    mkdir -p gpurun_out/r05k
    timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "brute" > gpurun_out/r05k/tests.log 2>&1 || exit 1
    for v in default abvar/lib_brh16.so abvar/lib_brg8.so abvar/lib_br2.so abvar/lib_brt1k.so; do
      if [ "$v" = default ]; then L=""; else L="RT_LIB=$v"; fi
      env $L timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05k/brute_$(basename $v .so).json 2> gpurun_out/r05k/brute_$(basename $v .so).err || exit 1
    done
    ;;
  r05l)
    # all configs with the CPU baseline, strong probes C4/C2
    mkdir -p gpurun_out/r05l
    timeout -k 10 900 python3 tools/bench_all.py --frames 20 --cpu-seconds 8 > gpurun_out/r05l/bench_all.jsonl 2> gpurun_out/r05l/bench_all.err || exit 1
    timeout -k 10 600 python3 tools/strong_probe.py --steps 20 --config c4_mixed --gather accumulation > gpurun_out/r05l/strong_c4_acc.jsonl 2> gpurun_out/r05l/strong_c4_acc.err || exit 1
    timeout -k 10 600 python3 tools/strong_probe.py --steps 20 --config c2_rtiow --gather accumulation > gpurun_out/r05l/strong_c2_acc.jsonl 2> gpurun_out/r05l/strong_c2_acc.err || exit 1
    ;;
  r05m)
    # refill prologue tests + A/B
    mkdir -p gpurun_out/r05m
    timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -x -v --timeout 120 --timeout-method thread -m gpu -k "golden or frame_batch or group or full_frame or sphere or determinism or camera or device" > gpurun_out/r05m/tests.log 2>&1 || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_noprep.so --config c2_rtiow --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/r05m/ab_c2.json 2> gpurun_out/r05m/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_noprep.so --config c1_four_spheres --width 800 --height 600 --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/r05m/ab_c1.json 2> gpurun_out/r05m/ab_c1.err || exit 1
    ;;
  r05n)
    # C5 regression check (ABI-11 commit build vs now, q4 compiled in/out)
    mkdir -p gpurun_out/r05n
    timeout -k 10 600 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_3e26.so abvar/lib_q4.so --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/r05n/ab_c5.json 2> gpurun_out/r05n/ab_c5.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_3e26.so --config c3_chess --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/r05n/ab_c3.json 2> gpurun_out/r05n/ab_c3.err || exit 1
    timeout -k 10 300 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_3e26.so --config c2_rtiow --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/r05n/ab_c2.json 2> gpurun_out/r05n/ab_c2.err || exit 1
    ;;
  r05o)
    # lazy triangle piece loads -- tests and A/B against the previous build
    mkdir -p gpurun_out/r05o
    timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "triangle or chess or golden or pruning or walk" > gpurun_out/r05o/tests.log 2>&1 || exit 1
    for c in c3_chess c4_mixed c5_heightfield; do
      timeout -k 10 300 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_nolazy.so abvar/lib_head.so --config $c --rounds 4 --frames 40 --frame-batch 20 > gpurun_out/r05o/ab_$c.json 2> gpurun_out/r05o/ab_$c.err || exit 1
    done
    ;;
  r05p)
    # lazy triangle pieces on C5, three builds in one process
    mkdir -p gpurun_out/r05p
    timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_nolazy.so abvar/lib_head.so --config c5_heightfield --rounds 4 --frames 40 --frame-batch 20 > gpurun_out/r05p/ab_c5.json 2> gpurun_out/r05p/ab_c5.err || exit 1
    ;;
  r05q)
    # streamed brute-force sweep variant
    mkdir -p gpurun_out/r05q
    RT_LIB=abvar/lib_bstream.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "brute" > gpurun_out/r05q/tests.log 2>&1 || exit 1
    timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05q/brute_default.json 2> gpurun_out/r05q/brute_default.err || exit 1
    RT_LIB=abvar/lib_bstream.so timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05q/brute_stream.json 2> gpurun_out/r05q/brute_stream.err || exit 1
    ;;
  r05r)
    # node pairs in the global-memory walk
    mkdir -p gpurun_out/r05r
    timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "heightfield or c5 or quantized or pruning or grazing or walk or certif or leaf or triangle_accel or device_scene" > gpurun_out/r05r/tests.log 2>&1 || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_nopairs.so abvar/lib_pairs_u3.so --config c5_heightfield --rounds 4 --frames 40 --frame-batch 20 > gpurun_out/r05r/ab_c5.json 2> gpurun_out/r05r/ab_c5.err || exit 1
    ;;
  r05s)
    # the whole GPU suite, smoke, headline bench
    mkdir -p gpurun_out/r05s
    timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05s/tests.log 2>&1 || exit 1
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05s/smoke.log 2>&1 || exit 1
    timeout -k 10 400 python3 bench.py > gpurun_out/r05s/bench.json 2> gpurun_out/r05s/bench.err || exit 1
    ;;
  r05t)
    # brute-force occupancy variants
    mkdir -p gpurun_out/r05t
    for v in default abvar/lib_bstream.so abvar/lib_bs_w6.so abvar/lib_bs_w8.so abvar/lib_bt_w6.so; do
      if [ "$v" = default ]; then L=""; else L="RT_LIB=$v"; fi
      env $L timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05t/brute_$(basename $v .so).json 2> gpurun_out/r05t/brute_$(basename $v .so).err || exit 1
    done
    ;;
  r05u)
    # brute-force modes (tiled / scalar-streamed)
    mkdir -p gpurun_out/r05u
    timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "brute" > gpurun_out/r05u/tests.log 2>&1 || exit 1
    timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05u/brute_tiled.json 2> gpurun_out/r05u/brute_tiled.err || exit 1
    timeout -k 10 200 python3 bench.py --config c5_heightfield --brute-force stream --steps 2 --warmup 1 --no-cpu-baseline --no-cadences > gpurun_out/r05u/brute_stream.json 2> gpurun_out/r05u/brute_stream.err || exit 1
    ;;
  r05v)
    # round-5 final profiles: kernel trace + PMC passes per bench line (tools/profile.sh)
    bash tools/profile.sh r05_c2 > gpurun_out/prof_r05_c2.log 2>&1 || exit 1
    bash tools/profile.sh r05_c5 --config c5_heightfield > gpurun_out/prof_r05_c5.log 2>&1 || exit 1
    bash tools/profile.sh r05_c3 --config c3_chess > gpurun_out/prof_r05_c3.log 2>&1 || exit 1
    bash tools/profile.sh r05_c4 --config c4_mixed --width 3840 --height 2160 > gpurun_out/prof_r05_c4.log 2>&1 || exit 1
    bash tools/profile.sh r05_c5b --config c5_heightfield --brute-force --steps 2 --warmup 2 > gpurun_out/prof_r05_c5b.log 2>&1 || exit 1
    bash tools/profile.sh r05_c5bs --config c5_heightfield --brute-force stream --steps 2 --warmup 2 > gpurun_out/prof_r05_c5bs.log 2>&1 || exit 1
    ;;
  r05w)
    # C5 knobs at the final build
    mkdir -p gpurun_out/r05w
    timeout -k 10 500 python3 tools/ab_env.py "RT_LEAF_BATCH=4" "RT_LEAF_BATCH=3" "RT_LEAF_BATCH=5" "RT_TRAV_THRESHOLD=48" "RT_TRAV_THRESHOLD=60" "RT_DRAIN_THRESHOLD=24" --config c5_heightfield --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05w/ab_knobs.jsonl 2> gpurun_out/r05w/ab_knobs.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_u4.so abvar/lib_u6.so --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/r05w/ab_unroll.json 2> gpurun_out/r05w/ab_unroll.err || exit 1
    ;;
  r05x)
    # scalar loads in the primary pre-pass -- tests, bench A/B
    mkdir -p gpurun_out/r05x
    timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "primary or heightfield or c5 or pruning or grazing or quantized or walk or full_size" > gpurun_out/r05x/tests.log 2>&1 || exit 1
    for i in 1 2; do
    timeout -k 10 200 python3 bench.py --config c5_heightfield --no-cpu-baseline --no-cadences > gpurun_out/r05x/c5_new_$i.json 2> gpurun_out/r05x/c5_new_$i.err || exit 1
    RT_LIB=abvar/lib_head.so timeout -k 10 200 python3 bench.py --config c5_heightfield --no-cpu-baseline --no-cadences > gpurun_out/r05x/c5_head_$i.json 2> gpurun_out/r05x/c5_head_$i.err || exit 1
    done
    ;;
  r05y)
    # sphere pair leaves (RT_SPHERE_PAIRS) -- parity and A/B
    mkdir -p gpurun_out/r05y
    RT_SPHERE_PAIRS=1 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_group.py -x -v --timeout 200 --timeout-method thread -m gpu -k "golden or full_frame or c2 or c1 or four_spheres or rtiow or sphere or brute or frame_batch" > gpurun_out/r05y/tests.log 2>&1 || exit 1
    timeout -k 10 500 python3 tools/ab_env.py "RT_SPHERE_PAIRS=0" "RT_SPHERE_PAIRS=1" "RT_SPHERE_PAIRS=1 RT_SPHERE_LEAF=1" --config c2_rtiow --frame-batch 20 --frames 40 --rounds 5 > gpurun_out/r05y/ab_c2.jsonl 2> gpurun_out/r05y/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_env.py "RT_SPHERE_PAIRS=0" "RT_SPHERE_PAIRS=1" --config c1_four_spheres --frame-batch 20 --frames 40 --rounds 5 > gpurun_out/r05y/ab_c1.jsonl 2> gpurun_out/r05y/ab_c1.err || exit 1
    ;;
  r05z)
    # round-5 final pass: the whole GPU suite, smoke, headline bench, profiles of every bench line
    mkdir -p gpurun_out/r05z
    timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05z/tests.log 2>&1 || exit 1
    RT_LIB=abvar/lib_q4.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "global_walk_variants" > gpurun_out/r05z/tests_q4.log 2>&1 || exit 1
    timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05z/smoke.log 2>&1 || exit 1
    timeout -k 10 400 python3 bench.py > gpurun_out/r05z/bench.json 2> gpurun_out/r05z/bench.err || exit 1
    bash tools/profile.sh r05f_c2 > gpurun_out/r05z/prof_c2.log 2>&1 || exit 1
    bash tools/profile.sh r05f_c5 --config c5_heightfield > gpurun_out/r05z/prof_c5.log 2>&1 || exit 1
    bash tools/profile.sh r05f_c3 --config c3_chess > gpurun_out/r05z/prof_c3.log 2>&1 || exit 1
    bash tools/profile.sh r05f_c4 --config c4_mixed --width 3840 --height 2160 > gpurun_out/r05z/prof_c4.log 2>&1 || exit 1
    bash tools/profile.sh r05f_c5b --config c5_heightfield --brute-force --steps 2 --warmup 2 > gpurun_out/r05z/prof_c5b.log 2>&1 || exit 1
    bash tools/profile.sh r05f_c5bs --config c5_heightfield --brute-force stream --steps 2 --warmup 2 > gpurun_out/r05z/prof_c5bs.log 2>&1 || exit 1
    ;;
  r05aa)
    # C3/C4 in the global-memory walk (mode 1) vs LDS-resident (mode 2)
    mkdir -p gpurun_out/r05aa
    timeout -k 10 400 python3 tools/ab_env.py "RT_LDS_MODE=2" "RT_LDS_MODE=1" "RT_LDS_MODE=1 RT_PRIMARY_PASS=0" --config c3_chess --frame-batch 20 --frames 40 --rounds 4 > gpurun_out/r05aa/ab_c3.jsonl 2> gpurun_out/r05aa/ab_c3.err || exit 1
    timeout -k 10 600 python3 tools/ab_env.py "RT_LDS_MODE=2" "RT_LDS_MODE=1" --config c4_mixed --width 3840 --height 2160 --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05aa/ab_c4.jsonl 2> gpurun_out/r05aa/ab_c4.err || exit 1
    ;;
  r05ab)
    # cooperative leaf batches in the LDS-resident walk (RT_COOP_LDS build)
    mkdir -p gpurun_out/r05ab
    RT_LIB=abvar/lib_cooplds.so timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "chess or c3 or c4 or mixed or golden or lds or full_frame" > gpurun_out/r05ab/tests.log 2>&1 || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_cooplds.so --config c3_chess --rounds 5 --frames 40 --frame-batch 20 > gpurun_out/r05ab/ab_c3.json 2> gpurun_out/r05ab/ab_c3.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_cooplds.so --config c4_mixed --width 3840 --height 2160 --rounds 3 --frames 20 --frame-batch 20 > gpurun_out/r05ab/ab_c4.json 2> gpurun_out/r05ab/ab_c4.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_cooplds.so --config c2_rtiow --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/r05ab/ab_c2.json 2> gpurun_out/r05ab/ab_c2.err || exit 1
    ;;
  r05ad)
    # strong-scaling probes at the final build: C2 with both payloads, C4 with the accumulation
    mkdir -p gpurun_out/r05ad
    timeout -k 10 600 python3 tools/strong_probe.py --steps 20 --config c2_rtiow --gather accumulation > gpurun_out/r05ad/strong_c2_accumulation.jsonl 2> gpurun_out/r05ad/strong_c2_accumulation.err || exit 1
    timeout -k 10 600 python3 tools/strong_probe.py --steps 20 --config c2_rtiow --gather image > gpurun_out/r05ad/strong_c2_image.jsonl 2> gpurun_out/r05ad/strong_c2_image.err || exit 1
    timeout -k 10 600 python3 tools/strong_probe.py --steps 20 --config c4_mixed --gather accumulation > gpurun_out/r05ad/strong_c4_accumulation.jsonl 2> gpurun_out/r05ad/strong_c4_accumulation.err || exit 1
    ;;
  r05ae)
    # small-subtree certificates (RT_TRI_SUBTREE) -- parity on the walks from global memory, C5 A/B
    mkdir -p gpurun_out/r05ae
    timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "heightfield or c5 or pruning or grazing or quantized or walk or certif" > gpurun_out/r05ae/tests.log 2>&1 || exit 1
    timeout -k 10 600 python3 tools/ab_env.py "RT_TRI_SUBTREE=0" "RT_TRI_SUBTREE=2" "RT_TRI_SUBTREE=3" "RT_TRI_SUBTREE=4" --config c5_heightfield --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05ae/ab_subtree.jsonl 2> gpurun_out/r05ae/ab_subtree.err || exit 1
    ;;
  r05af)
    # the same with the subtree tests deferred to the leaf batches (r05ae tested them on the spot)
    mkdir -p gpurun_out/r05af
    timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "heightfield or c5 or pruning or grazing or quantized or walk or certif" > gpurun_out/r05af/tests.log 2>&1 || exit 1
    timeout -k 10 600 python3 tools/ab_env.py "RT_TRI_SUBTREE=0" "RT_TRI_SUBTREE=2" "RT_TRI_SUBTREE=3" "RT_TRI_SUBTREE=4" --config c5_heightfield --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05af/ab_subtree.jsonl 2> gpurun_out/r05af/ab_subtree.err || exit 1
    ;;
  r05ag)
    # subtree tests deferred, the waiting lane marked through its node index -- parity, A/B against the
    # round's final build (abvar/lib_head.so) in one process, and the subtree sizes
    mkdir -p gpurun_out/r05ag
    timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "heightfield or c5 or pruning or grazing or quantized or walk or certif" > gpurun_out/r05ag/tests.log 2>&1 || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_head.so --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/r05ag/ab_head.json 2> gpurun_out/r05ag/ab_head.err || exit 1
    timeout -k 10 600 python3 tools/ab_env.py "RT_TRI_SUBTREE=0" "RT_TRI_SUBTREE=2" "RT_TRI_SUBTREE=4" --config c5_heightfield --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05ag/ab_subtree.jsonl 2> gpurun_out/r05ag/ab_subtree.err || exit 1
    ;;
  r05ah)
    # workgroup size at the final build: 1024 threads (4 waves per SIMD, 128 VGPRs with spills) against
    # 512 / 256 (3 waves per SIMD, no spills), on the triangle scenes
    mkdir -p gpurun_out/r05ah
    for c in c5_heightfield c3_chess c4_mixed; do
    timeout -k 10 400 python3 tools/ab_env.py "RT_BLOCK_THREADS=1024" "RT_BLOCK_THREADS=512" "RT_BLOCK_THREADS=256" --config $c --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05ah/ab_threads_$c.jsonl 2> gpurun_out/r05ah/ab_threads_$c.err || exit 1
    done
    ;;
  r05ai)
    # traversal knobs re-checked at the final build: C2, C3, C4 (at its 4K size)
    mkdir -p gpurun_out/r05ai
    timeout -k 10 300 python3 tools/ab_env.py "RT_TRAV_THRESHOLD=8" "RT_TRAV_THRESHOLD=6" "RT_TRAV_THRESHOLD=10" "RT_TRAV_THRESHOLD=12" --config c2_rtiow --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05ai/ab_c2.jsonl 2> gpurun_out/r05ai/ab_c2.err || exit 1
    timeout -k 10 300 python3 tools/ab_env.py "RT_TRAV_THRESHOLD=24" "RT_TRAV_THRESHOLD=16" "RT_TRAV_THRESHOLD=32" "RT_LEAF_BATCH=5" "RT_LEAF_BATCH=7" --config c3_chess --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05ai/ab_c3.jsonl 2> gpurun_out/r05ai/ab_c3.err || exit 1
    timeout -k 10 400 python3 tools/ab_env.py "RT_TRAV_THRESHOLD=24" "RT_TRAV_THRESHOLD=16" "RT_TRAV_THRESHOLD=32" "RT_LEAF_BATCH=5" "RT_LEAF_BATCH=7" --config c4_mixed --width 3840 --height 2160 --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05ai/ab_c4.jsonl 2> gpurun_out/r05ai/ab_c4.err || exit 1
    ;;
  r05ak)
    # the leaf batch's certificate and triangle-block loads non-temporal (abvar/lib_nt.so, -DRT_NT_LEAF=1):
    # do the node lines stay in the L1 longer?
    mkdir -p gpurun_out/r05ak
    timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_nt.so --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/r05ak/ab_nt.json 2> gpurun_out/r05ak/ab_nt.err || exit 1
    ;;
  r05al)
    # multi-frame packets in the primary pre-pass (RT_PRIMARY_FRAMES=2 / 4) -- parity, C5 A/B, F=1 against
    # the final build in one process
    mkdir -p gpurun_out/r05al
    RT_PRIMARY_FRAMES=4 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "primary or heightfield or c5 or pruning or grazing or quantized or walk or frame_batch" > gpurun_out/r05al/tests_f4.log 2>&1 || exit 1
    RT_PRIMARY_FRAMES=2 timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread -m gpu -k "primary or heightfield or c5 or pruning or grazing" > gpurun_out/r05al/tests_f2.log 2>&1 || exit 1
    timeout -k 10 600 python3 tools/ab_env.py "RT_PRIMARY_FRAMES=1" "RT_PRIMARY_FRAMES=2" "RT_PRIMARY_FRAMES=4" --config c5_heightfield --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05al/ab_frames.jsonl 2> gpurun_out/r05al/ab_frames.err || exit 1
    timeout -k 10 400 python3 tools/ab_bench.py rust_gpu_raytracing_amd/librt_pathtrace.so abvar/lib_head.so --config c5_heightfield --rounds 3 --frames 40 --frame-batch 20 > gpurun_out/r05al/ab_head.json 2> gpurun_out/r05al/ab_head.err || exit 1
    ;;
  r05am)
    # C3 / C4 scene-side knobs at the final build (sphere leaves and layouts, sub-object staging, claim order)
    mkdir -p gpurun_out/r05am
    K='"RT_SPHERE_LEAF=0" "RT_SPHERE_LEAF=2" "RT_SPHERE_LEAF=8" "RT_SPHERE_OCTANTS=0" "RT_SPHERE_BOX_ORDER=0" "RT_STAGE_SUBS=0" "RT_STAGE_SUBS=1" "RT_TILE_SCHEDULE=0" "RT_UNIT_TILE_MAJOR=0" "RT_UNIT_TILE_MAJOR=1" "RT_BATCH_SCHEDULE=1"'
    eval timeout -k 10 400 python3 tools/ab_env.py $K --config c4_mixed --width 3840 --height 2160 --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05am/ab_c4.jsonl 2> gpurun_out/r05am/ab_c4.err || exit 1
    eval timeout -k 10 300 python3 tools/ab_env.py $K --config c3_chess --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05am/ab_c3.jsonl 2> gpurun_out/r05am/ab_c3.err || exit 1
    ;;
  r05aj)
    # the TD-rate microbenchmark with its L1-hit and coalesced-line variants (build it first:
    # hipcc --offload-arch=gfx950 -O3 tools/microbench/td_rate.hip -o tools/microbench/td_rate)
    mkdir -p gpurun_out/r05aj
    timeout -k 10 120 ./tools/microbench/td_rate > gpurun_out/r05aj/td_rate.txt 2>&1 || exit 1
    ;;
  r05_verify)
    # end-of-session check of the committed tree: every GPU test, smoke, the headline bench
    bash tools/gpu_check.sh r05_verify tests smoke bench || exit 1
    ;;
  *) echo "unknown run $1"; exit 2 ;;
esac
