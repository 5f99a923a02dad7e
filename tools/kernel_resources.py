"""Per-kernel register and scratch usage of the built libblsgpu.so (gfx950), read from the code objects'
AMDGPU metadata notes: VGPRs, AGPRs, SGPRs, private segment (scratch) bytes per lane, LDS bytes, and the
waves per SIMD the register file allows.

    python tools/kernel_resources.py [lib.so] [--json out.json]

The .hip_fatbin section holds one offload bundle per translation unit; each is split out and unbundled with
clang-offload-bundler, then llvm-readelf --notes prints the metadata.  Host-only tooling (no GPU).
"""
import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def code_objects(lib):
    with tempfile.TemporaryDirectory() as td:
        fat = os.path.join(td, "fat.bin")
        subprocess.check_call([f"{LLVM}/llvm-objcopy", "-O", "binary", "--only-section=.hip_fatbin", lib, fat])
        data = open(fat, "rb").read()
        starts = [m.start() for m in re.finditer(re.escape(MAGIC), data)]
        for k, s in enumerate(starts):
            e = starts[k + 1] if k + 1 < len(starts) else len(data)
            b = os.path.join(td, f"b{k}.bin")
            open(b, "wb").write(data[s:e].rstrip(b"\0") if k + 1 == len(starts) else data[s:e])
            lst = subprocess.run([f"{LLVM}/clang-offload-bundler", "--list", "--type=o", f"--input={b}"],
                                 capture_output=True, text=True).stdout.split()
            tgt = [t for t in lst if "gfx" in t]
            if not tgt:
                continue
            co = os.path.join(td, f"b{k}.co")
            subprocess.check_call([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={b}",
                                   f"--targets={tgt[0]}", f"--output={co}"])
            yield subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], capture_output=True, text=True).stdout


FIELDS = {".vgpr_count": "vgpr", ".agpr_count": "agpr", ".sgpr_count": "sgpr",
          ".private_segment_fixed_size": "scratch_B", ".group_segment_fixed_size": "lds_B",
          ".vgpr_spill_count": "vgpr_spill", ".sgpr_spill_count": "sgpr_spill"}


def parse(notes):
    # amdhsa.kernels is a YAML list of maps with alphabetically ordered keys: a kernel's record starts at its
    # list item ("  - .agpr_count: ..."), and .agpr_count / .group_segment_fixed_size come BEFORE its .name
    out, cur = [], None
    for line in notes.splitlines():
        if re.match(r"^  - \.", line):
            cur = {}
            out.append(cur)
        s = line.strip().lstrip("- ").strip()
        m = re.match(r"(\.[a-z_]+):\s+(.*)$", s)
        if not m or cur is None:
            continue
        key, val = m.groups()
        if key == ".name" and not val.endswith(".kd") and line.startswith("    .name"):
            cur["kernel"] = val
        elif key in FIELDS and not line.startswith("      "):
            cur[FIELDS[key]] = int(val)
    out = [k for k in out if "kernel" in k]
    for k in out:
        # gfx950: 512 unified VGPR+AGPR entries per lane per SIMD, allocated in granules of 8; the metadata's
        # .vgpr_count is already the unified total (ArchVGPRs aligned + AGPRs), .agpr_count its AGPR part
        regs = (k.get("vgpr", 0) + 7) // 8 * 8
        k["waves_per_simd"] = min(8, 512 // max(regs, 1))
    return out


def main():
    args = [a for a in sys.argv[1:]]
    out_json = None
    if "--json" in args:
        i = args.index("--json")
        out_json = args[i + 1]
        del args[i:i + 2]
    lib = args[0] if args else os.path.join(os.path.dirname(__file__), "..", "lodestar_amd", "libblsgpu.so")
    ks = []
    for notes in code_objects(lib):
        ks += [k for k in parse(notes) if k.get("vgpr") is not None]
    ks.sort(key=lambda k: k["kernel"])
    print(f"{'kernel':40s} {'vgpr':>5s} {'agpr':>5s} {'sgpr':>5s} {'scratch':>8s} {'lds':>7s} {'w/SIMD':>6s}")
    for k in ks:
        print(f"{k['kernel'][:40]:40s} {k.get('vgpr', 0):5d} {k.get('agpr', 0):5d} {k.get('sgpr', 0):5d} "
              f"{k.get('scratch_B', 0):8d} {k.get('lds_B', 0):7d} {k['waves_per_simd']:6d}")
    if out_json:
        json.dump(ks, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main()
