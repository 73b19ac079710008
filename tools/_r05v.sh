# round-5 final profiles: kernel trace + PMC passes per bench line (tools/profile.sh)
set -o pipefail
bash tools/profile.sh r05_c2 > gpurun_out/prof_r05_c2.log 2>&1 || exit 1
bash tools/profile.sh r05_c5 --config c5_heightfield > gpurun_out/prof_r05_c5.log 2>&1 || exit 1
bash tools/profile.sh r05_c3 --config c3_chess > gpurun_out/prof_r05_c3.log 2>&1 || exit 1
bash tools/profile.sh r05_c4 --config c4_mixed --width 3840 --height 2160 > gpurun_out/prof_r05_c4.log 2>&1 || exit 1
bash tools/profile.sh r05_c5b --config c5_heightfield --brute-force --steps 2 --warmup 2 > gpurun_out/prof_r05_c5b.log 2>&1 || exit 1
bash tools/profile.sh r05_c5bs --config c5_heightfield --brute-force stream --steps 2 --warmup 2 > gpurun_out/prof_r05_c5bs.log 2>&1 || exit 1
