"""How sensitive is the REFERENCE's BRECQ act phase (block_recon.py:62-73, 400 iterations of
recon_brecq_long) to a one-ulp perturbation of its starting act deltas?  Runs the
reference twice on CPU (make_golden's loading recipe): as recorded in the fixture, and with
every act quantizer's delta nudged by one fp32 ulp before the act phase; writes the
divergence of the two reference trajectories (per-iteration losses, final deltas) as JSON.
This bounds what any other fp32 summation order (the GPU's convs) can be expected to match.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/brecq_sensitivity.py OUT.json"""
import json
import sys

import numpy as np
import torch

import make_golden as MG


def run(nudge):
    got = {}
    orig_save, orig_br = MG.save, MG.BR.block_reconstruction

    def save(name, **arrays):
        got.update(arrays)

    def br(qnn, block, *a, **k):
        if k.get("act_quant") and nudge:
            with torch.no_grad():
                for m in [block] + list(block.modules()):
                    q = getattr(m, "act_quantizer", None)
                    if q is not None and isinstance(getattr(q, "delta", None), torch.Tensor):
                        q.delta.copy_(torch.nextafter(q.delta, torch.full_like(q.delta, 1.0)))
        return orig_br(qnn, block, *a, **k)

    MG.save, MG.BR.block_reconstruction = save, br
    try:
        MG.gen_recon_brecq(iters=400, name="recon_brecq_long")
    finally:
        MG.save, MG.BR.block_reconstruction = orig_save, orig_br
    return got


if __name__ == "__main__":
    torch.set_num_threads(4)
    a, b = run(False), run(True)
    la, lb = a["a_total_loss"], b["a_total_loss"]
    rel = np.abs(la - lb) / np.abs(la)
    out = {"what": "reference BRECQ act phase, recon_brecq_long (400 iterations), run twice: "
                   "as recorded vs every act delta nudged by one fp32 ulp before the act phase",
           "weight_phase_identical": bool(np.array_equal(a["w_total_loss"], b["w_total_loss"])),
           "act_loss_rel_diff": {"iters_0_20_max": float(rel[:20].max()),
                                 "iters_0_100_max": float(rel[:100].max()),
                                 "max": float(rel.max()), "median": float(np.median(rel))},
           "act_loss_window_mean_rel_diff": [float(abs(la[i:i + 100].mean() - lb[i:i + 100].mean()) /
                                                   la[i:i + 100].mean()) for i in range(0, 400, 100)],
           "final_delta_rel_diff": (np.abs(a["a_delta"] - b["a_delta"]) / np.abs(a["a_delta"])).tolist()}
    json.dump(out, open(sys.argv[1], "w"), indent=1)
    print(json.dumps(out, indent=1))
