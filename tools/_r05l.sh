# round-5 session script (scratch): all configs with the CPU baseline, strong probes C4/C2
set -o pipefail
mkdir -p gpurun_out/r05l
timeout -k 10 900 python3 tools/bench_all.py --frames 20 --cpu-seconds 8 > gpurun_out/r05l/bench_all.jsonl 2> gpurun_out/r05l/bench_all.err || exit 1
timeout -k 10 600 python3 tools/strong_probe.py --steps 20 --config c4_mixed --gather accumulation > gpurun_out/r05l/strong_c4_acc.jsonl 2> gpurun_out/r05l/strong_c4_acc.err || exit 1
timeout -k 10 600 python3 tools/strong_probe.py --steps 20 --config c2_rtiow --gather accumulation > gpurun_out/r05l/strong_c2_acc.jsonl 2> gpurun_out/r05l/strong_c2_acc.err || exit 1
