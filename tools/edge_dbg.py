import os, sys
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/oracle"); sys.path.insert(0, "/root/repo/tests")
import cask_ref as R
from conftest import GOLDEN
import cask_amd
ctx = cask_amd.ScanContext(0)
case = os.path.join(GOLDEN, "edge_sizes")
files = [(f, open(R.data_file_path(case, f), "rb").read()) for f in R.find_data_files(case)]
print("files", [(f, len(b)) for f, b in files], flush=True)
res = ctx.scan_host(files)
print("count", res.count, "err", res.error, ctx.last_counters(), flush=True)
