"""CPU restatement of the fused shifted-scale reconstruction loop on a ResNet BasicBlock.

TEST INFRASTRUCTURE ONLY: tests/test_oracle.py pins it to the reference's own trajectory
(tests/golden/recon_fused.npz) and bench.py times it as the recon leg of `cpu_baseline`
("port": the reference's algorithm in plain PyTorch-CPU ops, run on the GPU box's host
cores).  The product path never imports this module.

What one iteration computes (block_recon_fused_shiftedScale,
/root/reference/quant/layer_recon_fused_shiftedScale.py:23-141):
  * batch = cached[torch.randperm(N)[:32]]                                        (:95-97)
  * per conv, ChannelQuant 'adaShift' (channelQuant.py:51-64, 96-118):
      x_q[i] = floor(W / (delta * s_i))  -- computed ONCE, as init_v_beta does (:284-286)
      p      = clamp(softmax(alpha) * (zeta - gamma) + gamma, 0, 1)               (:120-121)
      x_out  = x_q[0]*p0;  x_out += x_q[i]*p_i ...   (separate fp32 roundings)
      W_hat  = (clamp(x_out + h(beta) + zp, 0, n-1) - zp) * (delta * 1.0)
  * QuantBasicBlock.forward (quant_block.py:99-117) with QuantModule.forward's
    gamma^z/phi^z affine (quant_layer.py:245-280): relu(conv1) -> conv2 -> + residual -> relu
  * loss = lp(p=2) + [count >= 0.2*iters] * (lR*sum(1-|2h(beta)-1|^b) + lS*sum(1-|2p-1|^b2))
    (FusedScaleLossFunction, :223-309; schedules FusedLinearTempDecayShift :382-399)
  * backward, Adam(lr 1e-3) over alpha (+ gamma^z/phi^z with bias_cal).
The initialisation follows ChannelQuant.init_alpha / inverse_softmax / init_v_beta
(channelQuant.py:158-199, 279-294).
"""
import torch
import torch.nn.functional as F

GAMMA, ZETA = -0.1, 1.1


def _init_alpha(w, floors):
    """channelQuant.py:158-199 (clip forced to 0.33; per input channel for conv)."""
    S = len(floors)
    mse = torch.stack([torch.sum((w - xq) ** 2, dim=(0, 2, 3)) for xq in floors], dim=0)
    _, idx = torch.min(mse, dim=0)
    clip, rest = (1.0, 0.0) if S == 1 else (0.33, (1.0 - 0.33) / (S - 1))
    probs = torch.full((idx.shape[0], S), rest, dtype=torch.float)
    for i in range(S):
        probs[:, i][idx == i] = clip
    x = (probs - GAMMA) / (ZETA - GAMMA)
    logits = torch.log(x)
    return logits - torch.mean(logits, dim=-1, keepdim=True)


def _soft_targets(alpha):
    return torch.clamp(F.softmax(alpha, dim=-1) * (ZETA - GAMMA) + GAMMA, 0, 1)


class _Conv:
    def __init__(self, w, b, delta, zp, shifts, n_bits, stride, padding, bias_cal):
        self.w, self.b = w, b
        self.delta, self.zp = delta.view(-1, 1, 1, 1), zp.view(-1, 1, 1, 1)
        self.n_levels = 2 ** n_bits
        self.stride, self.padding = stride, padding
        self.floors = [torch.floor(w / (self.delta * s)) for s in shifts]       # x_q, once
        self.alpha = torch.nn.Parameter(_init_alpha(w, self.floors))
        p = _soft_targets(self.alpha)
        sel = torch.tensor(shifts)[torch.argmax(p, dim=-1)]                     # get_delta
        d_sel = self.delta * sel.view(1, -1, 1, 1)
        rest = w / d_sel - torch.floor(w / d_sel)
        self.beta = -torch.log((ZETA - GAMMA) / (rest - GAMMA) - 1)            # init_v_beta
        self.h = torch.clamp(torch.sigmoid(self.beta) * (ZETA - GAMMA) + GAMMA, 0, 1)
        co = w.shape[0]
        self.gamma_z = torch.nn.Parameter(torch.ones(1, co, 1, 1), requires_grad=bias_cal)
        self.phi_z = torch.nn.Parameter(torch.zeros(1, co, 1, 1), requires_grad=bias_cal)

    def what(self):
        p = _soft_targets(self.alpha).unsqueeze(0).unsqueeze(-1).unsqueeze(-1)
        x_out = self.floors[0] * p[:, :, 0, :, :]
        for i in range(1, len(self.floors)):
            x_out = x_out + self.floors[i] * p[:, :, i, :, :]
        q = torch.clamp(x_out + self.h + self.zp, 0, self.n_levels - 1)
        return (q - self.zp) * (self.delta * 1.0)

    def __call__(self, x):
        out = F.conv2d(x, self.what(), self.b, stride=self.stride, padding=self.padding)
        return out * self.gamma_z + self.phi_z


class FusedBlockReconCPU:
    """The loop above for one QuantBasicBlock; `convs` maps 'conv1'/'conv2'/['downsample']
    to (weight, bias, delta, zero_point, stride, padding)."""

    def __init__(self, convs, shifts, n_bits, cached_inp, cached_out, iters, lmda=(0.01, 0.1),
                 bias_cal=False, batch_size=32):
        self.convs = {k: _Conv(*v[:4], shifts, n_bits, v[4], v[5], bias_cal) for k, v in convs.items()}
        params = [c.alpha for c in self.convs.values()]
        if bias_cal:
            params += [t for c in self.convs.values() for t in (c.gamma_z, c.phi_z)]
        self.opt = torch.optim.Adam(params, lr=1e-3)
        self.inp, self.out = cached_inp, cached_out
        self.bs = batch_size
        self.lR, self.lS = lmda
        self.iters = iters
        self.count = 0
        self.loss_start = iters * 0.2

    def _decay(self, t_max):
        """FusedLinearTempDecayShift(t_max, rel_start_decay=0.2, 20 -> 2) at self.count."""
        start = 0.2 * t_max
        if self.count < start:
            return 20
        rel = (self.count - start) / (t_max - start) if t_max != 0 else 1
        return 2 + (20 - 2) * max(0.0, 1 - rel)

    def block(self, x):
        c = self.convs
        residual = x if 'downsample' not in c else c['downsample'](x)
        out = F.relu(c['conv1'](x))
        out = c['conv2'](out)
        out = out + residual
        return F.relu(out)

    def step(self):
        """One iteration; returns the reconstruction loss."""
        perm = torch.randperm(self.inp.size(0))[:self.bs]
        inp, tgt = self.inp[perm], self.out[perm]
        self.opt.zero_grad()
        pred = self.block(inp)
        rec = (pred - tgt).abs().pow(2.0).sum(1).mean()
        total = rec
        b, b2 = self._decay(self.iters), self._decay(self.iters * 3 / 4)
        if self.count >= self.loss_start:
            for c in self.convs.values():
                total = total + self.lR * (1 - ((c.h - .5).abs() * 2).pow(b)).sum()
                ps = _soft_targets(c.alpha)
                total = total + self.lS * (1 - ((ps - .5).abs() * 2).pow(b2)).sum()
        total.backward()
        self.opt.step()
        self.count += 1
        return float(rec.detach())
