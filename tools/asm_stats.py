#!/usr/bin/env python3
"""Static instruction mix of transport_kernel<true> (device asm via hipcc -S); no GPU needed.
usage: asm_stats.py [extra hipcc flags...]"""
import collections
import re
import subprocess
import sys

src = "/root/repo/rsmcrt_amd/csrc/smcrt.hip"
subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math",
                "--offload-arch=gfx950", "--cuda-device-only", "-S", "-o", "/tmp/smcrt_stats.s", src] + sys.argv[1:],
               check=True, cwd="/tmp", stderr=subprocess.DEVNULL)
s = open("/tmp/smcrt_stats.s").read()
m = re.search(r"^(_Z16transport_kernelILb1E\w+):", s, re.M)
start = m.start()
end = s.index(".Lfunc_end", start)
ins = [l.strip() for l in s[start:end].splitlines()]
ins = [l for l in ins if l and not l.startswith((".", ";", "_")) and not l.endswith(":")]
c = collections.Counter(i.split()[0] for i in ins)
valu = sum(v for k, v in c.items() if k.startswith("v_"))
print(f"total {len(ins)}  valu {valu}  salu {sum(v for k, v in c.items() if k.startswith('s_'))}  "
      f"readlane {c['v_readlane_b32']}  writelane {c['v_writelane_b32']}  div {c['v_div_fixup_f64']}  "
      f"sqrt {c['v_sqrt_f64_e32']}  ds {sum(v for k, v in c.items() if k.startswith('ds_'))}  "
      f"global {sum(v for k, v in c.items() if k.startswith('global_'))}")
for k, v in c.most_common(int(dict(enumerate(sys.argv)).get(99, 0) or 0)):
    print(k, v)
