"""Print the kernel times of kprof JSON files: python tools/show_kprof.py FILE_OR_DIR..."""
import glob
import json
import os
import sys

for arg in sys.argv[1:]:
    files = sorted(glob.glob(os.path.join(arg, "*.json"))) if os.path.isdir(arg) else [arg]
    for f in files:
        try:
            d = json.load(open(f))
        except Exception as e:  # noqa: BLE001
            print(f, "unreadable:", e)
            continue
        parts = [f"{k}={v['ms_median']}ms" for k, v in d.items() if isinstance(v, dict) and "ms_median" in v]
        print(f, " ".join(parts))
