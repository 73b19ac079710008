# round-5 session script (scratch): the whole GPU suite, smoke, headline bench
set -o pipefail
mkdir -p gpurun_out/r05s
timeout -k 10 1100 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r05s/tests.log 2>&1 || exit 1
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05s/smoke.log 2>&1 || exit 1
timeout -k 10 400 python3 bench.py > gpurun_out/r05s/bench.json 2> gpurun_out/r05s/bench.err || exit 1
