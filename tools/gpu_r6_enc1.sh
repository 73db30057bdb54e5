# round 6: the first layer on the limb MFMA -- encoder fp64 / golden / sharding tests, then the A/B
export TMPDIR=/tmp
O=gpurun_out/${1:-r6j}; mkdir -p $O
timeout -k 10 300 python -u tools/enc_ab.py DAMC_ENC_FIRST_MFMA 1,0 celebaHQ:64 celebaHQ:8 celeba64:256 celeba64:32 > $O/enc_ab.txt 2>&1
rc=$?; cat $O/enc_ab.txt | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu -k "encoder or xemb or celebaHQ_q or amortizer or checkpoint" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; exit $rc
