export TMPDIR=/tmp
O=gpurun_out/r05_agree; mkdir -p $O
timeout -k 10 900 python -u tools/agreement.py --c4 0 --c5 0 --host-c4 10000000 --out $O/host_c4.json > $O/host_c4.log 2>&1 || { tail -30 $O/host_c4.log; exit 1; }
tail -2 $O/host_c4.log
