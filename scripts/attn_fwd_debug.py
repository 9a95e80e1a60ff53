"""Direct call of edl_attn_fwd with NaN-filled outputs: which parts does the kernel write, how wrong."""
import json
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from easydl_amd import _native  # noqa: E402


def run(var, mode, B=1, S=64, H=2, KV=1, causal=1):
    os.environ["EDL_ATTN_FWD"], os.environ["EDL_ATTN_FWD_MODE"] = var, mode
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(B, S, H, 128, device="cuda", generator=g).bfloat16()
    k = torch.randn(B, S, KV, 128, device="cuda", generator=g).bfloat16()
    v = torch.randn(B, S, KV, 128, device="cuda", generator=g).bfloat16()
    o = torch.full_like(q, float("nan"))
    lse = torch.full((B, H, S), float("nan"), device="cuda")
    _native.kernels().check("edl_attn_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                            B, S, H, KV, 128, causal, 1 / math.sqrt(128), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    kk = k.float().repeat_interleave(H // KV, dim=2)
    vv = v.float().repeat_interleave(H // KV, dim=2)
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), kk) / math.sqrt(128)
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device="cuda"), 1), float("-inf"))
    ref_lse = torch.logsumexp(s, -1)
    ref_o = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), vv)
    of = o.float()
    return {"var": var + "m" + mode, "o_nan_frac": of.isnan().float().mean().item(),
            "o_absmax": of.nan_to_num(0).abs().max().item(), "ref_absmax": ref_o.abs().max().item(),
            "lse_nan_frac": lse.isnan().float().mean().item(),
            "lse_err": (lse - ref_lse).abs().nan_to_num(1e9).max().item(),
            "o_row0": of[0, 0, 0, :6].tolist(), "ref_row0": ref_o[0, 0, 0, :6].tolist(),
            "o_row40": of[0, 40, 1, :4].tolist(), "ref_row40": ref_o[0, 40, 1, :4].tolist(),
            "lse_first": lse[0, 0, :4].tolist(), "ref_lse_first": ref_lse[0, 0, :4].tolist(),
            "lse_nan_rows": [[h_, r] for h_ in range(H) for r in range(S) if math.isnan(lse[0, h_, r].item())][:8],
            "lse_ok_rows": [[h_, r, round(lse[0, h_, r].item(), 3), round(ref_lse[0, h_, r].item(), 3)]
                            for h_ in range(H) for r in range(S) if not math.isnan(lse[0, h_, r].item())][:12],
            "o_zero_rows": sum(1 for h_ in range(H) for r in range(S) if of[0, r, h_].abs().max().item() == 0),
            "o_match_rows": sum(1 for h_ in range(H) for r in range(S)
                                if (of[0, r, h_] - ref_o[0, r, h_]).abs().max().item() < 2e-2)}


def dump(mode, S=64, H=2, KV=1):
    """MODE 8: wave 0 of block 0 writes m, l, raw/exp'd S and packed P after the prologue."""
    os.environ["EDL_ATTN_FWD"], os.environ["EDL_ATTN_FWD_MODE"] = "64", mode
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(1, S, H, 128, device="cuda", generator=g).bfloat16()
    k = torch.randn(1, S, KV, 128, device="cuda", generator=g).bfloat16()
    v = torch.randn(1, S, KV, 128, device="cuda", generator=g).bfloat16()
    o = torch.zeros_like(q)
    dbg = torch.full((64 * 64 + 4096,), float("nan"), device="cuda")
    _native.kernels().check("edl_attn_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), dbg.data_ptr(),
                            1, S, H, KV, 128, 1, 1 / math.sqrt(128), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    d = dbg[:4096].view(64, 64).cpu()
    s = (q[0, :, 0].float() @ k[0, :, 0].float().t()).cpu() / math.sqrt(128) * 1.4426950408889634
    out = []
    for lane in (0, 1, 4, 5, 32, 36):
        q_ = lane & 31
        h = lane >> 5
        keys = [(i & 3) + 8 * (i >> 2) + 4 * h for i in range(16)]
        out.append({"lane": lane, "m": d[lane, 0].item(), "ls": d[lane, 1].item(),
                    "ref_m": s[q_, :q_ + 1].max().item(),
                    "p_t0": [round(x, 3) for x in d[lane, 8:24].tolist()],
                    "raw_ref_t0": [round(s[q_, kk].item(), 3) if kk <= q_ else None for kk in keys],
                    "pb": d[lane, 40:48].tolist()})
    return out


def rows(mode, S=128, H=2, KV=1, causal=1):
    os.environ["EDL_ATTN_FWD"], os.environ["EDL_ATTN_FWD_MODE"] = "64", mode
    g = torch.Generator(device="cuda").manual_seed(0)
    q = torch.randn(1, S, H, 128, device="cuda", generator=g).bfloat16()
    k = torch.randn(1, S, KV, 128, device="cuda", generator=g).bfloat16()
    v = torch.randn(1, S, KV, 128, device="cuda", generator=g).bfloat16()
    o = torch.full_like(q, float("nan"))
    lse = torch.full((1, H, S), float("nan"), device="cuda")
    _native.kernels().check("edl_attn_fwd", q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), lse.data_ptr(),
                            1, S, H, KV, 128, causal, 1 / math.sqrt(128), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    kk, vv = k.float(), v.float()
    s = torch.einsum("bqhd,bkhd->bhqk", q.float(), kk.expand(-1, -1, H, -1)) / math.sqrt(128)
    if causal:
        s = s.masked_fill(torch.triu(torch.ones(S, S, dtype=torch.bool, device="cuda"), 1), float("-inf"))
    ref_lse = torch.logsumexp(s, -1)
    ref_o = torch.einsum("bhqk,bkhd->bqhd", torch.softmax(s, -1), vv.expand(-1, -1, H, -1))
    bad_o = [(h_, r) for h_ in range(H) for r in range(S)
             if (o[0, r, h_].float() - ref_o[0, r, h_]).abs().max().item() > 2e-2]
    bad_l = [(h_, r) for h_ in range(H) for r in range(S) if abs(lse[0, h_, r].item() - ref_lse[0, h_, r].item()) > 1e-3]
    bad_d = sorted({d for (h_, r) in bad_o[:4] for d in range(128)
                    if abs(o[0, r, h_, d].item() - ref_o[0, r, h_, d].item()) > 2e-2})
    return {"mode": mode, "n_bad_o": len(bad_o), "bad_o": bad_o[:40], "n_bad_lse": len(bad_l), "bad_lse": bad_l[:10],
            "bad_d_of_first_rows": bad_d[:64]}


if __name__ == "__main__":
    for m in ("2", "4"):
        print(json.dumps(rows(m)), flush=True)
    for var, mode in (("0", "0"), ("64", "0"), ("64", "6")):
        print(json.dumps(run(var, mode)), flush=True)
