"""The plain-C oracle (bench.py's CPU port) against the reference's golden vectors."""
import numpy as np

from oracle import c_oracle as CO


def test_c_oracle_uaq_golden(golden):
    g = golden("uaq")
    n = 0
    for k in g:
        if not k.endswith("_gdelta"):
            continue
        t = k[:-len("_gdelta")]
        bits = int(t.split("_")[0][1:])
        sym, cw, method = "_sym_" in t, "_cw_" in t, t.rsplit("_", 1)[1]
        x = g[t + "_x"]
        d, z, r = CO.init_scale(x, bits, sym, cw, method)
        np.testing.assert_array_equal(d, g[t + "_delta"], err_msg=t)
        np.testing.assert_array_equal(z, g[t + "_zp"], err_msg=t)
        y, _ = CO.fake_quant(x, d, z, bits, sym)
        np.testing.assert_array_equal(y, g[t + "_y"], err_msg=t)
        n += 1
    assert n >= 16
