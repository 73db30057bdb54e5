# CelebA-HQ B=8 (config 5 per rank of 8) under rocprofv3 --kernel-trace: per-dispatch grid and duration
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg
timeout -s KILL 300 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg/trace -o run --output-format csv -- python3 tools/cfg_profile.py _netG_celebaHQ 128 128 256 8 3 > gpurun_out/cfg/log.txt 2>&1 || exit 1
grep "per posterior" gpurun_out/cfg/log.txt
