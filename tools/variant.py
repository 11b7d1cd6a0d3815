"""Build an A/B variant of libpcs.so from a text patch of one source (timing experiments only:
the shipped sources carry no ablation switches).

    python tools/variant.py tools/variants/<spec>.py [more specs ...]

A spec defines NAME, SRC (e.g. "gemm_glds") and EDITS = [(old, new), ...]; each old must occur
exactly once in csrc/SRC.hip (or in that file as committed at REV, if the spec sets REV).  The variant goes to abtest/NAME/libpcs.so (select it with
PCS_LIB=abtest/NAME/libpcs.so), linked with the in-tree objects of every other source."""
import os
import runpy
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "point-cloud-cnn-segmentation_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-Wall", "-Wno-unused-function"]
EXTRA = {"gemm_glds": ["-mllvm", "-disable-machine-sink"], "gram_glds": ["-mllvm", "-disable-machine-sink"],
         "fused_seg4": ["-fno-slp-vectorize"], "fwd_s12": ["-fno-slp-vectorize"]}


def build(spec_path):
    spec = runpy.run_path(spec_path)
    name, src, edits = spec["NAME"], spec["SRC"], spec.get("EDITS", [])
    if spec.get("REV"):   # the source as committed at REV (e.g. the baseline of an A/B)
        rel = os.path.relpath(os.path.join(CSRC, src + ".hip"), REPO)
        text = subprocess.run(["git", "-C", REPO, "show", f"{spec['REV']}:{rel}"], check=True,
                              capture_output=True, text=True).stdout
    else:
        text = open(os.path.join(CSRC, src + ".hip")).read()
    for old, new in edits:
        n = text.count(old)
        if n != 1:
            raise SystemExit(f"{spec_path}: edit occurs {n} times: {old[:80]!r}")
        text = text.replace(old, new)
    out = os.path.join(REPO, "abtest", name)
    os.makedirs(out, exist_ok=True)
    hip = os.path.join(CSRC, f"_variant_{name}_{src}.hip")   # beside common.h for the includes
    open(hip, "w").write(text)
    obj = os.path.join(out, src + ".o")
    try:
        subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *EXTRA.get(src, []), "-c", hip, "-o", obj], check=True)
    finally:
        os.remove(hip)
    objs = [os.path.join(CSRC, f) for f in sorted(os.listdir(CSRC)) if f.endswith(".o") and f != src + ".o"]
    subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                    os.path.join(out, "libpcs.so"), obj, *objs], check=True)
    print("built", os.path.join(out, "libpcs.so"))


if __name__ == "__main__":
    subprocess.run(["make", "-C", CSRC, "-j8"], check=True, stdout=subprocess.DEVNULL)
    for p in sys.argv[1:]:
        build(p)
