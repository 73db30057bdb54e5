# round 5: the encoder's host time per call, then the CelebA-HQ encoder profile
export TMPDIR=/tmp
O=gpurun_out/${1:-r5he}; mkdir -p $O
timeout -k 10 120 python tools/enc_hosttime.py cifar10 128 50 2>/dev/null | tee $O/enc_hosttime.txt || exit 1
bash tools/gpu_r5_hqenc.sh ${1:-r5he}
