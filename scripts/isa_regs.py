"""Per-kernel register, spill and LDS figures from a hipcc -S listing
(raytracing2-fork_amd/build/rt2_render.s, `make isa`), with the number of
scratch stores / loads and SGPR-lane spills in each kernel's body.

    python scripts/isa_regs.py [listing] [--match SUBSTR]
"""
import argparse
import re
import sys


def kernels(text):
    """{symbol: metadata dict} from the listing's .amdgpu_metadata block."""
    out = {}
    for blk in re.split(r"\n\s+- \.agpr_count:", text):
        m = re.search(r"\.name:\s+(\S+)", blk)
        if not m:
            continue
        d = {"name": m.group(1)}
        for key in ("vgpr_count", "vgpr_spill_count", "sgpr_count", "sgpr_spill_count",
                    "group_segment_fixed_size", "private_segment_fixed_size"):
            k = re.search(r"\." + key + r":\s+(\d+)", blk)
            if k:
                d[key] = int(k.group(1))
        out[d["name"]] = d
    return out


def body_counts(text, sym):
    start = text.find("\n" + sym + ":")
    if start < 0:
        return {}
    end = text.find("s_endpgm", start)
    end = text.find("\n.Lfunc_end", start) if end < 0 else text.find("\n.Lfunc_end", end)
    body = text[start:end]
    return {"scratch_st": len(re.findall(r"scratch_store", body)),
            "scratch_ld": len(re.findall(r"scratch_load", body)),
            "writelane": len(re.findall(r"v_writelane", body)),
            "readlane": len(re.findall(r"v_readlane", body)),
            "mfma": len(re.findall(r"v_mfma", body))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("listing", nargs="?", default="raytracing2-fork_amd/build/rt2_render.s")
    ap.add_argument("--match", default="render_mfma")
    a = ap.parse_args()
    text = open(a.listing).read()
    for sym, d in kernels(text).items():
        if a.match not in sym:
            continue
        c = body_counts(text, sym)
        short = sym[-90:]
        print(f"{short}\n  vgpr {d.get('vgpr_count')} spill {d.get('vgpr_spill_count')} sgpr {d.get('sgpr_count')} "
              f"sgpr_spill {d.get('sgpr_spill_count')} lds {d.get('group_segment_fixed_size')} "
              f"scratch {d.get('private_segment_fixed_size')} | {c}")


if __name__ == "__main__":
    sys.exit(main())
