"""ssq_lp_loss's one-launch form (SSQ_LOSS_ONE_LAUNCH=1, read once per process, hence a
process of its own) on two streams at once: tests/test_kernels_gpu.py
test_lp_loss_one_launch_two_streams.

Each stream's calls get their own workspace (kernels.workspace keys on the stream), and
the last-arriver counter lives in that workspace (csrc/recon.hip lp_loss_ticket), so two
reductions in flight never count each other's workgroups: every loss value and gradient
equals the one-stream result bit for bit, over repeated rounds (the counter resets).

    SSQ_LOSS_ONE_LAUNCH=1 python tests/lp_loss_streams_worker.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    assert os.environ.get("SSQ_LOSS_ONE_LAUNCH") == "1"
    from shiftedscalequantization_amd import kernels as K
    gen = torch.Generator().manual_seed(77)
    # 1024 workgroups apiece (the launch's cap): both grids fill the chip together
    preds = [torch.randn(64, 256, 28, 28, generator=gen).cuda() for _ in range(2)]
    tgts = [torch.randn(64, 256, 28, 28, generator=gen).cuda() for _ in range(2)]

    def run(i, p):
        loss, g = K.lp_loss_and_grad(preds[i], tgts[i], p)
        return loss, g

    def bits(r):
        return [t.detach().cpu().numpy().reshape(-1).view(np.int32).copy() for t in r]

    for p in (2.0, 2.4):
        base = []
        for i in range(2):
            r = run(i, p)
            torch.cuda.synchronize()
            base.append(bits(r))
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        for _ in range(16):
            res = []
            for i in range(2):
                with torch.cuda.stream(streams[i]):
                    res.append(run(i, p))
            torch.cuda.synchronize()
            for i in range(2):
                for a, b in zip(bits(res[i]), base[i]):
                    np.testing.assert_array_equal(a, b)
        # the float64 truth of the value: the one-launch sum is the partials in index order
        for i in range(2):
            ref = (preds[i] - tgts[i]).double().abs().pow(p).sum(1).mean().item()
            got = float(base[i][0].view(np.float32)[0])
            # p = 2.4: hardware log2 / exp2 per term (csrc/ssq_common.h lp_term, ~1e-6)
            assert abs(got - ref) <= (1e-6 if p == 2.0 else 1e-5) * abs(ref), (p, got, ref)
    print("LP_LOSS_STREAMS_OK")


if __name__ == "__main__":
    main()
