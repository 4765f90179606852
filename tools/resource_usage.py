"""Print VGPRs / SGPRs / scratch / LDS per kernel of libdqrm (hipcc -Rpass-analysis)."""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
src = f"{ROOT}/deep_quantized_recommendation_model_dqrm_amd/csrc/dqrm_kernels.hip"
cmd = ["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared", "-ffp-contract=off",
       f"-I{ROOT}/include", "-Rpass-analysis=kernel-resource-usage", src, "-o", "/tmp/_ru.so"] + sys.argv[1:]
out = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = {}
for line in out.splitlines():
    m = re.search(r"remark: Function Name: (\S+)", line)
    if m:
        cur = m.group(1)
        rows[cur] = {}
        continue
    m = re.search(r"remark:\s+(VGPRs|TotalSGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]): (\d+)", line)
    if m and cur:
        rows[cur][m.group(1).split()[0]] = int(m.group(2))
for k, v in rows.items():
    name = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", k)
    print(f"{name[:60]:60s} vgpr={v.get('VGPRs')} sgpr={v.get('TotalSGPRs')} scratch={v.get('ScratchSize')} occ={v.get('Occupancy')}")
