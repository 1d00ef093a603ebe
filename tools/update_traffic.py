"""Refresh one config's entry of profiles/traffic.json from a tools/profile_c2.sh summary:

    python3 tools/update_traffic.py profiles/r03/r03y/c2/summary.json c2 1000000

traffic = HBM bytes per signature stage (FETCH_SIZE x 2 + WRITE_SIZE of the stage's kernels over
the run / the stage executions; bench.py --no-extra runs, so there are no other launches), the form bench.py
reads into roofline.traffic (it checks units and the kernel description)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main(summary, config, units):
    import bench  # the kernel description bench.py matches on
    d = json.load(open(summary))
    st = d["stages"]["ecdsa" if config in ("c2", "c3", "c4") else "schnorr"]
    path = os.path.join(ROOT, "profiles", "traffic.json")
    tj = json.load(open(path))
    e = tj.get(config, {})
    # per stage = all launches of the stage's kernels / the stage executions of the run (a stage
    # launches its kernels once per lane chunk: C4's 8M tuples are two 4M chunks)
    e.update(units=units, traffic_bytes=st["traffic_bytes"],
             fetch_bytes_x2=st["fetch_bytes_x2"], write_bytes=st["write_bytes"],
             source=f"{os.path.relpath(summary, ROOT)} (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes "
                    f"over bench.py --no-extra, {st['executions']} stage executions of "
                    f"{', '.join(st['kernels'])}; FETCH doubled per MI355X_MICROARCH.md)",
             kernel=bench.ECDSA_KERNELS if config in ("c2", "c3", "c4") else bench.SCHNORR_KERNELS)
    e.pop("instruction_mix", None)
    tj[config] = e
    json.dump(tj, open(path, "w"), indent=1)
    print(json.dumps(e, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]))
