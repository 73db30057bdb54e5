export TMPDIR=/tmp
for d in 0 31; do echo "dbg=$d"; DAMC_CHAIN_DBG=$d timeout -k 10 300 python tools/sweep_profile.py 128 2>&1 | grep -v amdgpu.ids; done
