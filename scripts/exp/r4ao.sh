# Breakout PPO: weight-gradient plane counts (conv2/conv3 nhwc_planes, conv1_planes) -- fewer planes = fewer bytes
# written by the wgrad kernels and read by the finaliser, but fewer workgroups.
set -o pipefail
for o in '{}' '{"nhwc_planes": 128}' '{"nhwc_planes": 64}' '{"conv1_planes": 64}' '{"nhwc_planes": 128, "conv1_planes": 64}' '{}'; do
  timeout -k 10 300 python -u scripts/bench_configs.py --configs breakout_ppo --updates 5 --warmup 2 --engine-opts "$o" | cut -c1-110 || exit 1
  echo "  opts $o"
done
