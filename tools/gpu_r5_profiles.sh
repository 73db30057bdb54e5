export TMPDIR=/tmp
O=gpurun_out/r5c; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/b16 -o run --output-format csv -- python3 tools/b16_profile.py 16 > $O/b16.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/svhn -o run --output-format csv -- python3 tools/cfg_profile.py _netG_svhn 100 64 32 64 > $O/svhn.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/qup -o run --output-format csv -- python3 tools/q_update_trace.py 5 > $O/qup.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $O/enc -o run --output-format csv -- python3 tools/encoder_profile.py cifar10 128 5 > $O/enc.log 2>&1 || exit 1
for v in "" "DAMC_ENC_WSRC=0" "DAMC_ENC_F32A=0" "DAMC_ENC_IN_SLABS=0" "" "DAMC_ENC_WSRC=0" "DAMC_ENC_F32A=0" "DAMC_ENC_IN_SLABS=0"; do
  echo "[$v] $(env $v timeout -k 5 60 python3 tools/encoder_profile.py cifar10 128 20 2>&1 | tail -1)" >> $O/enc_ab.txt || exit 1
done
