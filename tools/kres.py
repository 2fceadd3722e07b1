"""Kernel resources from hipcc -Rpass-analysis=kernel-resource-usage output: python3 tools/kres.py A.txt [B.txt]
(prints every sqp_step_kernel instantiation's VGPR/AGPR/scratch; with two files, only those that differ)."""
import re
import subprocess
import sys


def parse(f):
    out, cur = {}, None
    for line in open(f):
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            out[cur] = {}
            continue
        m = re.search(r"remark:\s+(VGPRs|AGPRs|ScratchSize \[bytes/lane\]|VGPRs Spill|TotalSGPRs): (\d+)", line)
        if m and cur:
            out[cur][m.group(1).split()[0]] = int(m.group(2))
    return out


a = parse(sys.argv[1])
b = parse(sys.argv[2]) if len(sys.argv) > 2 else None
for k in a:
    if "sqp_step" not in k or (b is not None and a[k] == b.get(k)):
        continue
    n = subprocess.run(["c++filt", k], capture_output=True, text=True).stdout.strip()
    n = n.replace("void gpmpc::sqp_step_kernel", "").split("(")[0]
    print(n, a[k], "" if b is None else b.get(k))
