# driver-style 20-step bench with per-iteration clock / power / last-collective attribution
set -o pipefail
mkdir -p gpurun_out/r6d
B=$(python3 -c "import glob;print(' '.join(glob.glob('/sys/bus/pci/devices/*/hwmon/hwmon*/freq1_input')[:2]))" || true)
echo "freq1_input: $B" > gpurun_out/r6d/sensors.txt
timeout -k 10 1000 python -u bench.py --steps 20 --warmup 1 > gpurun_out/r6d/bench.log 2> gpurun_out/r6d/bench.err
