# round-5 session script (scratch): PMC of the C5 walk (TCP/TA/TD) and of the brute-force wavefront
set -o pipefail
bash tools/pmc_tcp.sh r05_c5tcp --config c5_heightfield || exit 1
bash tools/profile.sh r05_c5b --config c5_heightfield --brute-force --steps 2 --warmup 2 || exit 1
