"""Build an alternative engine library with extra -D flags into
microbench/_variants/<name>.so (load it with SPEEDB_AMD_LIB=...)."""
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
name, defs = sys.argv[1], sys.argv[2:]
out = os.path.join(REPO, "microbench", "_variants", name + ".so")
os.makedirs(os.path.dirname(out), exist_ok=True)
csrc = os.path.join(REPO, "speedb_amd", "csrc")
subprocess.check_call(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-shared",
                       "-Wall", "-Wno-unused-function"] + ["-D" + d for d in defs] +
                      ["-o", out] + [os.path.join(csrc, f) for f in
                                     ("mck_engine.hip", "mck_sst.cc", "mck_blob.cc", "mck_wal.cc", "mck_walrec.cc")])
print(out)
