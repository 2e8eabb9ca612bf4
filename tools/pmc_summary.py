"""Per-kernel averages of every counter in rocprofv3 --pmc pass directories.

    python tools/pmc_summary.py <pass_dir> [<pass_dir> ...]
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main():
    vals = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as fp:
                for row in csv.DictReader(fp):
                    name = row.get("Kernel_Name", "")
                    short = name.replace("rt::(anonymous namespace)::", "").split("(")[0]
                    vals[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items() if "kd3" in k or "trace" in k}
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
