# round 6: CIFAR encoder call with the weight packing as separate launches (DAMC_ENC_WSRC=0): how much of the first
# layer's launch is the merged packing
export TMPDIR=/tmp
O=gpurun_out/${1:-r6ep}; mkdir -p $O
DAMC_ENC_WSRC=0 timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/enc -o run --output-format csv -- python3 tools/encoder_profile.py cifar10 128 3 > $O/enc.log 2>&1 || exit 1
f=$(find $O/enc -name '*kernel_trace.csv' | head -1)
python3 tools/trace_tail.py $f "pack_conv|conv3_" "cifar10 encoder B=128 (DAMC_ENC_WSRC=0): one call" | tee $O/enc_dispatches.txt
