"""Average rocprofv3 --pmc counters per dispatch, per kernel (substring match).

    python tools/pmc_summary.py <dir with *counter_collection.csv> [kernel_substring]

Every pass directory also holds lib.sha256, the sha256 of the libwcsde.so the profiled process
ran (written by the pass script on the GPU box); lib_stamp() checks that all passes of one summary
agree and returns it, and bench.py attaches a profiles/pmc_*.json only when its stamp equals the
sha256 of the library it has loaded.
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


def lib_stamp(*dirs):
    """The sha256 of the library the passes in `dirs` ran (their lib.sha256 files), all equal."""
    stamps = set()
    for d in dirs:
        f = os.path.join(d, "lib.sha256")
        if not os.path.exists(f):
            raise RuntimeError(f"{f} missing: the pass predates the library stamp; run it again")
        stamps.add(open(f).read().split()[0])
    if len(stamps) != 1:
        raise RuntimeError(f"passes ran different libraries: {sorted(stamps)}")
    return stamps.pop()


if __name__ == "__main__":
    print(json.dumps(summary(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None), indent=1))
