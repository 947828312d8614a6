"""Average rocprofv3 --pmc counters per dispatch, per kernel (substring match).

    python tools/pmc_summary.py <dir with *counter_collection.csv> [kernel_substring]
"""
import collections
import csv
import glob
import json
import os
import sys


def summary(d, sub=None):
    out = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.defaultdict(set)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if sub and sub not in k:
                continue
            key = k.replace("void ", "").replace("(anonymous namespace)::", "").split("((")[0][:100]
            out[key][r["Counter_Name"]] += float(r["Counter_Value"])
            n[key].add(r.get("Dispatch_Id", r.get("Correlation_Id")))
    return {k: {c: v / max(1, len(n[k])) for c, v in cs.items()} | {"dispatches": len(n[k])} for k, cs in out.items()}


if __name__ == "__main__":
    print(json.dumps(summary(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None), indent=1))
