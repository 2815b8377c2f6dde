# host-path bench only (pinned / pageable / API encode + API host-file prove)
mkdir -p gpurun_out/r3c
timeout -k 10 500 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-parity-sample --host-path > gpurun_out/r3c/bench_host.json 2> gpurun_out/r3c/bench_host.err; rc=$?
tail -c 1500 gpurun_out/r3c/bench_host.json; tail -5 gpurun_out/r3c/bench_host.err; exit $rc
