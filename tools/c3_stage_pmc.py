"""The C3 roofline stage alone, for rocprofv3 counter passes: bench.py's C3 workload (4000
block-413567-shaped txs, seed 0x5EED0003), its first round staged in HBM, the sighash stage once and
then the ECDSA stage (bench.py C3.kernel_times' run_ecdsa) REPS times, nothing else on the GPU
afterwards.  tools/gpu_c3_traffic.sh runs it under FETCH_SIZE / WRITE_SIZE passes and divides the
stage kernels' bytes by REPS (+ the wl.run() execution)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "rust-bitcoinconsensus_amd"))
import bench  # noqa: E402
import bitcoinconsensus_amd as B  # noqa: E402

REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 10
job = bench.C3(B, bench.DEFAULT_N["c3"], bench.SEEDS["c3"], 0)
job.wl.run()  # one full staged round (sighash + ECDSA): messages in place
for _ in range(REPS):
    job.wl.run_ecdsa(None)
job.wl.verdicts()
print(f"c3 staged ECDSA stage x{REPS + 1}: {job.shape['tuples']} tuples", flush=True)
