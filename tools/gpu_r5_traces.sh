# round 5 end: dispatch traces of one CIFAR B=16 and one SVHN B=64 posterior step on HEAD
export TMPDIR=/tmp
O=gpurun_out/${1:-r5tr}; mkdir -p $O
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/svhn -o run --output-format csv -- python3 tools/cfg_profile.py _netG_svhn 100 64 32 64 > $O/svhn.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace -d $O/b16 -o run --output-format csv -- python3 tools/b16_profile.py 16 > $O/b16.log 2>&1 || exit 1
ls -R $O | head -20
