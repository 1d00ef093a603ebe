#!/bin/bash
# Pipelining A/B on the box (run via gpurun): the drop-in verify_batch over 1M C2 inputs per
# pipeline chunk (tools/e2e_pipe.py), then bcc_pubkey_verify_batch over the C4 set per part size
# (bench.py --config c4's drop_in_end_to_end).  usage: tools/gpu_pipe_ab.sh TAG
export TMPDIR=/tmp
O=gpurun_out/${1:-pipe}
mkdir -p $O
timeout -k 10 300 python -u tools/e2e_pipe.py 1000000 10 2 0 131072 262144 500000 > $O/e2e_pipe.txt 2>&1 || { tail -20 $O/e2e_pipe.txt; exit 1; }
cat $O/e2e_pipe.txt
for p in 0 1048576 2097152; do
    BCC_PIPELINE_CHUNK=$p timeout -k 10 300 python3 bench.py --config c4 --no-cpu --steps 5 --warmup 2 --sustain-s 0 > $O/c4_part$p.json 2> $O/c4_part$p.err || { tail -20 $O/c4_part$p.err; exit 2; }
    python3 -c "import json; d=json.load(open('$O/c4_part$p.json')); e=d['drop_in_end_to_end']; print('c4 part $p', round(e['verifies_per_s']/1e6,2), 'M/s', round(e['ms'],1), 'ms', e['mismatches_vs_staged'])"
done
