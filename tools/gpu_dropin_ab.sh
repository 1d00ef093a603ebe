# Interleaved A/B of the drop-in (tools/dropin_e2e.py: best call, 20 sustained calls, phases)
# over environment settings, one process per setting and round.
#   tools/gpu_dropin_ab.sh TAG ROUNDS "VAR=a" "VAR=b" ...
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:?tag}; R=${2:-3}; shift 2
mkdir -p $O
for rep in $(seq 1 $R); do
  for s in "$@"; do
    timeout -k 10 200 env PHASES=1 $s python3 tools/dropin_e2e.py 1000000 20 2>&1 | grep -v amdgpu.ids >> $O/ab.txt || { tail -5 $O/ab.txt; exit 1; }
  done
done
python3 - $O/ab.txt <<'PY'
import ast, re, sys, collections
rows = collections.defaultdict(list)
lines = open(sys.argv[1]).read().splitlines()
for i, ln in enumerate(lines):
    m = re.match(r"(\{.*?\}) threads=.*sustained ([\d.]+) M/s, ([\d.]+) CPU-s", ln)
    if m:
        env = ast.literal_eval(m.group(1))
        mem = env.pop("mem_GBps", None)
        ph = re.search(r"interpret=([\d.]+)", lines[i + 1]) if i + 1 < len(lines) else None
        rows[str(env)].append((float(m.group(2)), float(m.group(3)), float(ph.group(1)) if ph else None, mem))
for k, v in rows.items():
    print(k, "sustained", [x[0] for x in v], "cpu_s/M", [x[1] for x in v], "interpret_ms",
          [x[2] for x in v], "mem_GBps", [x[3] for x in v])
PY
