"""Print value / ms_per_step of the bench JSON line in each given gpu_run log (missing: '-')."""
import json
import sys

for path in sys.argv[1:]:
    try:
        line = [ln for ln in open(path) if ln.startswith('{"metric"')][-1]
        d = json.loads(line)
        print(path, d["value"], d["ms_per_step"])
    except (OSError, IndexError, ValueError):
        print(path, "-")
