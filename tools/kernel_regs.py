"""Summarise hipcc -Rpass-analysis=kernel-resource-usage remarks (VGPR/AGPR/spill/occupancy)."""
import re
import sys

OCC = re.compile(r"Occupancy \[waves/SIMD\]: (\d+)")


def main(paths, filt=""):
    for path in paths:
        txt = open(path).read()
        for b in txt.split("Function Name: ")[1:]:
            name = b.split(" ")[0]
            if filt and not re.search(filt, name):
                continue
            g = {k: re.search(k + r": (\d+)", b).group(1) for k in ("VGPRs", "AGPRs", "VGPRs Spill")}
            print(f"{name[:90]:90s} V={g['VGPRs']} A={g['AGPRs']} spill={g['VGPRs Spill']} occ={OCC.search(b).group(1)}")


if __name__ == "__main__":
    main(sys.argv[2:], sys.argv[1])
