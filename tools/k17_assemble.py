"""Assemble conv_wgrad.hip from the new stage-1 source (/tmp/k17_stage1.hip) and HEAD's
stage 2 / depthwise kernels / entry points, with the new planner and launch; patch the
Python gate and the K17 parity cases.  (One-off build step of the K17 rewrite.)"""
import subprocess

R = "/root/repo/"
old = subprocess.run(["git", "-C", R, "show", "HEAD:shiftedscalequantization_amd/csrc/conv_wgrad.hip"],
                     capture_output=True, text=True, check=True).stdout
new = open("/tmp/k17_stage1.hip").read()
a = old.index("// dW = the splits summed in a fixed order")
b = old.index("static int wgrad_plan(")
helpers = old[a:b]
c = old.index("}  // namespace ssq")
entries = old[c:]
plan = r'''static size_t wgrad_lds(int wm, int pq, int64_t xtile) {
  return sizeof(float) * (2 * (size_t)(64 * wm) * (pq + 1) + 2 * (size_t)(xtile + 1));
}

static int wgrad_plan(int64_t Nb, int64_t C, int64_t H, int64_t W, int64_t Co, int64_t R,
                      int64_t S, int64_t st, int64_t pad, int64_t G, WgradGeo& g,
                      size_t* lds_bytes) {
  SSQ_REQUIRE(Nb >= 1 && C >= 1 && H >= 1 && W >= 1 && Co >= 1 && R >= 1 && S >= 1 && st >= 1 &&
                  pad >= 0 && G >= 1 && C % G == 0 && Co % G == 0,
              SSQ_E_ARG, "ssq_conv_wgrad: bad geometry");
  const int64_t OH = (H + 2 * pad - R) / st + 1, OW = (W + 2 * pad - S) / st + 1;
  SSQ_REQUIRE(OH >= 1 && OW >= 1 && Nb * C * H * W < (1ll << 31) && Nb * Co * OH * OW < (1ll << 31),
              SSQ_E_ARG, "ssq_conv_wgrad: sizes");
  g.Nb = (int)Nb; g.C = (int)C; g.H = (int)H; g.W = (int)W; g.Co = (int)Co;
  g.OH = (int)OH; g.OW = (int)OW; g.R = (int)R; g.S = (int)S; g.st = (int)st; g.pad = (int)pad;
  g.G = (int)G; g.Cig = (int)(C / G); g.Cog = (int)(Co / G);
  g.Ncol = g.Cig * g.R * g.S;
  const int RS = g.R * g.S;
  const int64_t Wp = W + 2 * pad;
  // Candidate layouts WM = 1, 2, 4 (TM = 64 WM, TN = 256 / WM) x Pq = 128, 64, in MFMA
  // slots (64 cycles): every tile runs 2 MFMAs per pixel per wave, plus per chunk a fixed
  // ~40 and one slot per LDS-DMA instruction a wave issues (A rows + x rows, / 4 waves).
  double best = 1e300;
  for (int wm : {1, 2, 4}) {
    for (int pq : {128, 64}) {
      const int TM = 64 * wm, TN = 256 / wm;
      const int64_t span = std::min<int64_t>(g.Cig, (TN - 1) / RS + 2);
      const int64_t orows = (pq - 1 + OW - 1) / OW + 1;     // output rows a chunk can span
      const int64_t in_rows = (orows - 1) * st + R;
      const int64_t xtile = span * in_rows * Wp;
      if (wgrad_lds(wm, pq, xtile) > 160 * 1024) continue;
      const int64_t cpn = (OH * OW + pq - 1) / pq;
      const int64_t tiles = ((g.Cog + TM - 1) / TM) * ((g.Ncol + TN - 1) / TN);
      const double dma = (double)(std::min<int64_t>(TM, g.Cog) * ((pq + 63) / 64) +
                                  span * in_rows * ((W + 63) / 64)) / 4.0;
      const double cost = (double)tiles * Nb * (2.0 * OH * OW + cpn * (40.0 + dma));
      if (cost < best) {
        best = cost;
        g.WM = wm;
        g.Pq = pq;
        g.ci_span = (int)span;
        g.in_rows = (int)in_rows;
        g.xtile = (int)xtile;
      }
    }
  }
  SSQ_REQUIRE(best < 1e300, SSQ_E_ARG, "ssq_conv_wgrad: input rows too wide for the LDS tile");
  const int TM = 64 * g.WM, TN = 256 / g.WM;
  g.lda = g.Pq + 1;
  g.chunks_per_n = (int)((OH * OW + g.Pq - 1) / g.Pq);
  g.nchunks = g.Nb * g.chunks_per_n;
  g.m_tiles = (g.Cog + TM - 1) / TM;
  g.n_tiles = (g.Ncol + TN - 1) / TN;
  const int64_t tiles = (int64_t)g.n_tiles * g.m_tiles * g.G;
  // about two workgroups per CU over the grid, at least 2 chunks each
  int nsplit = (int)std::max<int64_t>(1, std::min<int64_t>(g.nchunks / 2, (512 + tiles - 1) / tiles));
  g.cps = (g.nchunks + nsplit - 1) / nsplit;
  g.nsplit = (g.nchunks + g.cps - 1) / g.cps;
  *lds_bytes = wgrad_lds(g.WM, g.Pq, g.xtile);
  return SSQ_OK;
}

'''
i = entries.index("  static bool lds_attr = false;")
j = entries.index("  const int64_t n = (int64_t)Co * g.Ncol;")
launch = '''  static bool lds_attr = false;
  if (!lds_attr) {  // dynamic LDS beyond 64 KiB must be opted into
    hipFuncSetAttribute((const void*)wgrad_stage1<1>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    hipFuncSetAttribute((const void*)wgrad_stage1<2>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    hipFuncSetAttribute((const void*)wgrad_stage1<4>, hipFuncAttributeMaxDynamicSharedMemorySize,
                        160 * 1024);
    lds_attr = true;
  }
  const dim3 grid(g.n_tiles, g.m_tiles * g.G, g.nsplit);
  if (g.WM == 1)
    hipLaunchKernelGGL(wgrad_stage1<1>, grid, dim3(256), lds, s, x, dy, g, (float*)ws);
  else if (g.WM == 2)
    hipLaunchKernelGGL(wgrad_stage1<2>, grid, dim3(256), lds, s, x, dy, g, (float*)ws);
  else
    hipLaunchKernelGGL(wgrad_stage1<4>, grid, dim3(256), lds, s, x, dy, g, (float*)ws);
'''
entries = entries[:i] + launch + entries[j:]
open(R + "shiftedscalequantization_amd/csrc/conv_wgrad.hip", "w").write(new + "\n" + helpers + plan + entries)

p = R + "shiftedscalequantization_amd/kernels.py"
s = open(p).read()
s = s.replace('''    """Shapes ssq_conv_wgrad handles: 4-D fp32 NCHW on the device, square stride /
    padding, dilation 1, output width <= 128."""''', '''    """Shapes ssq_conv_wgrad handles: 4-D fp32 NCHW on the device, square stride /
    padding, dilation 1, and a plan whose LDS tile fits (nonzero workspace size)."""''')
s = s.replace('''    ow = (x.shape[3] + 2 * pad - weight.shape[3]) // st + 1
    return 1 <= ow <= 128
''', '''    Nb, C, H, W = (int(v) for v in x.shape)
    Co, _, R, S = (int(v) for v in weight.shape)
    return query("ssq_conv_wgrad_workspace_size", Nb, C, H, W, Co, R, S, int(st), int(pad),
                 int(groups)) > 0
''')
open(p, "w").write(s)
p = R + "tests/test_kernels_gpu.py"
s = open(p).read()
if "(2, 16, 14, 256, 1, 1, 0, 1)" not in s:
    s = s.replace('''    (1, 3, 32, 16, 7, 2, 3, 1),
    # depthwise path''', '''    (1, 3, 32, 16, 7, 2, 3, 1),
    # GEMM path layouts: few input channels (WM = 4 tiles), rows wider than a wave and than
    # a chunk, 7x7 planes (short chunks), stride 2 at 28x28
    (2, 16, 14, 256, 1, 1, 0, 1), (1, 8, 70, 16, 3, 1, 1, 1), (1, 4, 130, 8, 3, 1, 1, 1),
    (2, 256, 7, 512, 3, 1, 1, 1), (2, 64, 28, 128, 3, 2, 1, 1),
    # depthwise path''')
    open(p, "w").write(s)
print("assembled")
