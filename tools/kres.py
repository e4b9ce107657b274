"""Kernel resource summary from hipcc -Rpass-analysis=kernel-resource-usage output (not product).

    hipcc ... -Rpass-analysis=kernel-resource-usage 2> res.txt; python tools/kres.py res.txt [substring]
"""
import re
import subprocess
import sys


def main():
    text = open(sys.argv[1]).read().splitlines()
    pat = sys.argv[2] if len(sys.argv) > 2 else "ompl_amd"
    cur, out = None, []
    for ln in text:
        m = re.search(r"Function Name: (\S+)", ln)
        if m:
            cur = {"name": m.group(1)}
            out.append(cur)
            continue
        m = re.search(r"remark: ([A-Za-z ]+?): (\d+)", ln)
        if m and cur is not None:
            cur[m.group(1).strip()] = int(m.group(2))
    for k in out:
        if pat not in k["name"] or "target_arch" in k["name"]:
            continue
        try:
            dem = subprocess.run(["c++filt", k["name"]], capture_output=True, text=True).stdout.strip()
        except OSError:
            dem = k["name"]
        dem = re.sub(r"\(.*", "", dem.replace("ompl_amd::(anonymous namespace)::", ""))
        print(f"{dem[:70]:70s} vgpr {k.get('VGPRs', '?'):>3} agpr {k.get('AGPRs', '?'):>3} "
              f"sgpr {k.get('SGPRs', '?'):>3} scratch {k.get('ScratchSize [bytes/lane]', '?'):>4} "
              f"occ {k.get('Occupancy [waves/SIMD]', '?')} lds {k.get('LDS Size [bytes/block]', '?')}")


if __name__ == "__main__":
    main()
