# round-5 session script (scratch): C3/C4 in the global-memory walk (mode 1) vs LDS-resident (mode 2)
set -o pipefail
mkdir -p gpurun_out/r05aa
timeout -k 10 400 python3 tools/ab_env.py "RT_LDS_MODE=2" "RT_LDS_MODE=1" "RT_LDS_MODE=1 RT_PRIMARY_PASS=0" --config c3_chess --frame-batch 20 --frames 40 --rounds 4 > gpurun_out/r05aa/ab_c3.jsonl 2> gpurun_out/r05aa/ab_c3.err || exit 1
timeout -k 10 600 python3 tools/ab_env.py "RT_LDS_MODE=2" "RT_LDS_MODE=1" --config c4_mixed --width 3840 --height 2160 --frame-batch 20 --frames 20 --rounds 3 > gpurun_out/r05aa/ab_c4.jsonl 2> gpurun_out/r05aa/ab_c4.err || exit 1
