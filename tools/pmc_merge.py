#!/usr/bin/env python3
"""Merge the per-key PMC summaries a session wrote (pmc_traffic_<key>.json,
session.sh's pmcsum) into profiles/pmc_traffic.json.

    python tools/pmc_merge.py gpurun_out/<tag> [--copy profiles/r05/pmc_traffic]
"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

if __name__ == "__main__":
    src = sys.argv[1]
    copy = sys.argv[sys.argv.index("--copy") + 1] if "--copy" in sys.argv else None
    main = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    data = json.load(open(main)) if os.path.exists(main) else {}
    for f in sorted(glob.glob(os.path.join(src, "pmc_traffic_*.json"))):
        d = json.load(open(f))
        data.update(d)
        print(f, {k: v.get("build_id", "")[:8] for k, v in d.items()})
        if copy:
            shutil.copy(f, os.path.join(copy, os.path.basename(f)))
    with open(main, "w") as fp:
        json.dump(data, fp, indent=1, sort_keys=True)
