"""Diagnostic: the golden cases' rows through a given library build (tools only), host and device
scans, in the current CASK_SCAN_MODE. python tools/golden_check.py [LIB]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def main():
    import numpy as np
    import torch
    import cask_amd
    if len(sys.argv) > 1:
        cask_amd._lib.use_library(sys.argv[1])
    import cask_ref as R
    gold = os.path.join(ROOT, "tests", "golden")
    ctx = cask_amd.ScanContext(0)
    bad = 0
    for case in sorted(os.listdir(gold)):
        ej = os.path.join(gold, case, "expected.json")
        if not os.path.exists(ej):
            continue
        exp = json.load(open(ej))
        files = []
        for fe in exp["files"]:
            with open(R.data_file_path(os.path.join(gold, case), fe["file_id"]), "rb") as f:
                files.append((fe["file_id"], f.read()))
        for how in ("host", "device"):
            if how == "host":
                res = ctx.scan_host(files)
                get = lambda a, i: int(a[i])
            else:
                tens = [(fid, torch.from_numpy(np.frombuffer(b, np.uint8).copy()).cuda()) for fid, b in files]
                res = ctx.scan_device(tens)
                get = lambda a, i: int(a[i].item())
            for k, fe in enumerate(exp["files"]):
                sl = res.file_rows(k)
                got = [[get(res.pos, i), get(res.seq, i) & (2**64 - 1), get(res.ksz, i) & 0xFFFF,
                        get(res.vsz, i) & 0xFFFFFFFF, get(res.status, i)] for i in range(sl.start, sl.stop)]
                want = [r[:5] for r in fe["rows"]]
                if got != want:
                    bad += 1
                    j = next((j for j in range(min(len(got), len(want))) if got[j] != want[j]), None)
                    print("MISMATCH", case, how, fe["file_id"], len(got), len(want), j,
                          got[j] if j is not None else None, want[j] if j is not None else None)
    print("bad", bad, "walk", ctx.last_counters()["walk_mode"])


if __name__ == "__main__":
    main()
