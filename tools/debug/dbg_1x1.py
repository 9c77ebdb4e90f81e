import numpy as np, torch, sys, os
sys.path.insert(0, os.getcwd())
from oracle import ssq_ref as R
from shiftedscalequantization_amd import kernels as K
S = [31/32, 33/32, 1.0]
for shape in [(32, 16, 1, 1), (8, 6, 3, 3), (64, 64, 3, 3), (32, 16, 3, 3)]:
    g = torch.Generator().manual_seed(1)
    w = (torch.randn(shape, generator=g) * 0.05).numpy()
    d, z, _ = R.init_scale(w, 2, False, True, "max")
    xq, alpha, beta = R.init_v_beta(w, d, S)
    alpha = alpha + np.random.RandomState(0).randn(*alpha.shape).astype(np.float32) * 0.3
    gy = np.random.RandomState(1).randn(*shape).astype(np.float32)
    ga_ref, _ = R.adashift_bwd(xq, alpha, beta, d, z, 2, False, False, False, gy)
    a = torch.tensor(alpha).cuda().requires_grad_(True)
    y = K.adashift(a, torch.tensor(beta).cuda(), torch.tensor(w).cuda(), torch.tensor(d).cuda(), torch.tensor(z).cuda(), S, 2, False, False, False)
    y.backward(torch.tensor(gy).cuda())
    ga = a.grad.cpu().numpy()
    print(shape, "max abs err", np.abs(ga - ga_ref).max(), "max |g|", np.abs(ga_ref).max())
