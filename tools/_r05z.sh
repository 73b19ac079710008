# round-5 final pass: the whole GPU suite, smoke, headline bench, profiles of every bench line
set -o pipefail
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
