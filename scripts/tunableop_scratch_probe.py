"""Does a process read TunableOp's scratch results file, and can an entry in it break a GEMM?
(Round 6: ops/gemm_tuning.py pointed every process's output file at ONE per-user path; TunableOp
reads that file when it starts, and the "bogus" run failed its GEMM with "Expected iter !=
ops_.end()".  The output file is per process now: "bogus" must run the GEMM.)

  python scripts/tunableop_scratch_probe.py write   # apply(), one GEMM, exit: is the file written?
  python scripts/tunableop_scratch_probe.py bogus   # scratch holds an invalid solution index for
                                                    # a 512^3 GEMM: apply(), run that GEMM
"""
import os
import sys
import tempfile

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd.ops import gemm_tuning  # noqa: E402

SCRATCH = os.path.join(tempfile.gettempdir(), f"edl_tunableop_scratch_{os.getuid()}.csv")   # the old shared name


def show(tag):
    if os.path.exists(SCRATCH):
        txt = open(SCRATCH).read()
        print(f"[{tag}] scratch {len(txt)} bytes:\n{txt}", flush=True)
    else:
        print(f"[{tag}] no scratch file", flush=True)


mode = sys.argv[1]
if mode == "bogus":
    head = [ln for ln in open(gemm_tuning.SELECT_FILE).read().splitlines() if ln.startswith("Validator")]
    with open(SCRATCH, "w") as f:
        bad = "GemmTunableOp_BFloat16_NN,nn_512_512_512_ld_512_512_512,Gemm_Hipblaslt_7,0.01"
        f.write("\n".join(head + [bad]) + "\n")
show("before apply")
print("mode", gemm_tuning.apply(), flush=True)
show("after apply")
a = torch.randn(512, 512, device="cuda", dtype=torch.bfloat16)
c = a @ a
torch.cuda.synchronize()
print("gemm ok", float(c.float().abs().sum()) > 0, flush=True)
print("results", [r for r in torch.cuda.tunable.get_results()][:4], flush=True)
show("after gemm")
if mode == "bogus":
    os.unlink(SCRATCH)
