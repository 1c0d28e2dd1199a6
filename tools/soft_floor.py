"""The soft values' fp32 floor, on the CPU: for the seven cases
(transmitted offset / NCO phase) of test_demod_nco_matches_oracle (the same streams, frames and NCO-mixed samples),
max |q - q_oracle| over every soft value of 3 frames x 75 symbols when the FFT is
  gpu-emu      the GPU demod's radix-8/8/8/4 transform (tests/gpu_fft_emu.py)
  radix-4      the oracle's fp32 radix-4 Stockham transform (orc_fft2048_f32)
  r2-dit/dif   the oracle's fp32 radix-2 DIT / DIF transforms
against the oracle's double-precision FFT rounded to float; plus each transform's relative
rms error on random input and the count of soft values off by more than 1e-5.
usage: python tools/soft_floor.py > profiles/r06_soft_floor.txt"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "sdr-j-dab_amd"), os.path.join(ROOT, "tests"), os.path.join(ROOT, "tools")]
import dabamd                                    # noqa: E402
import gpu_fft_emu                               # noqa: E402
import oracle_py as orc                          # noqa: E402
from test_gpu_parity import NCO_CASES, _cfo_frames, _nco_mix   # noqa: E402

osc = dabamd.host_table(dabamd.TABLE_OSC)
mp = dabamd.host_table(dabamd.TABLE_MAPPER).astype(np.int64)
cb = np.where(mp < 0, mp + 2048, mp)
KINDS = {"radix-4": 1, "r2-dit": 2, "r2-dif": 3}


def q_of(X, P):
    """processToken's soft values (ofdm-decoder.cpp:180-189) in float: r = X conj(P), -re/L1, -im/L1"""
    Xr, Xi, Pr, Pi = [a.astype(np.float32) for a in (X[cb].real, X[cb].imag, P[cb].real, P[cb].imag)]
    rr = (Xr * Pr).astype(np.float32) - (Xi * (-Pi)).astype(np.float32)
    ri = (Xr * (-Pi)).astype(np.float32) + (Xi * Pr).astype(np.float32)
    ab = (np.abs(rr) + np.abs(ri)).astype(np.float32)
    return np.concatenate([(-rr / ab).astype(np.float32), (-ri / ab).astype(np.float32)])


def ffts(syms, kind):
    return np.array([(lambda y: y[0::2] + 1j * y[1::2])(orc.fft(np.stack([s.real, s.imag], 1).reshape(-1), 0, kind))
                     for s in syms])


def main():
    rng = np.random.default_rng(1)
    x = (rng.normal(size=(200, 2048)) + 1j * rng.normal(size=(200, 2048))).astype(np.complex64)
    ref = np.fft.fft(x.astype(np.complex128))
    print("relative rms error of the 2048-point transform (200 random complex Gaussian vectors):")
    rel = lambda X: np.sqrt(np.mean(np.abs(X - ref) ** 2) / np.mean(np.abs(ref) ** 2))
    print(f"  gpu-emu {rel(gpu_fft_emu.gpu_fft(x)):.3e}   double->f32 {rel(ffts(x, 0)):.3e}   " +
          "   ".join(f"{k} {rel(ffts(x, v)):.3e}" for k, v in KINDS.items()))
    print()
    print("max |q - q_oracle| (unweighted) per case (transmitted offset / NCO phase + data-symbol phase offset),")
    print("and [soft values off by > 1e-5], the rms, and round 6's criterion against the radix-4:")
    print(f"  {'cfo/nco':>14} " + " ".join(f"{k:>20}" for k in ["gpu-emu"] + list(KINDS)))
    cases = NCO_CASES
    for cfo, nco, off in cases:
        g, xs, frs = _cfo_frames(cfo, nco=nco, phase_b_off=off)
        res = {k: [0.0, 0, 0.0, 0] for k in ["gpu-emu"] + list(KINDS)}
        for fr in frs:
            pa = np.arange(fr.block0, fr.block0 + 2048)
            blk = _nco_mix(xs[pa], pa, fr.lp_window, fr.phase_a, fr.window, osc)
            dorg = fr.block0 + 2048
            pb = np.arange(dorg, dorg + 75 * 2552)
            seg = _nco_mix(xs[pb], pb, fr.lp_data, fr.phase_b, dorg, osc)
            syms = np.array([blk[:, 0] + 1j * blk[:, 1]] +
                            [seg[(l - 1) * 2552 + 504:l * 2552, 0] + 1j * seg[(l - 1) * 2552 + 504:l * 2552, 1]
                             for l in range(1, 76)]).astype(np.complex64)
            Xd = ffts(syms, 0)
            Xs = {"gpu-emu": gpu_fft_emu.gpu_fft(syms)}
            Xs.update({k: ffts(syms, v) for k, v in KINDS.items()})
            for l in range(1, 76):
                qd = q_of(Xd[l], Xd[l - 1])
                for k, X in Xs.items():
                    d = np.abs(q_of(X[l], X[l - 1]) - qd)
                    res[k][0] = max(res[k][0], float(d.max()))
                    res[k][1] += int((d > 1e-5).sum())
                    res[k][2] += float(np.sum(d.astype(np.float64) ** 2))
                    res[k][3] += d.size
        print(f"  {cfo:6.0f}/{nco if nco is not None else round(cfo):6.0f}+{off:<2d}" + " ".join(f"{v[0]:11.3e} [{v[1]:5d}]" for v in res.values()))
        rms = {k: np.sqrt(v[2] / v[3]) for k, v in res.items()}
        g, r4 = res["gpu-emu"], res["radix-4"]
        ok = (rms["gpu-emu"] <= 1.1 * rms["radix-4"], g[1] <= 2 * r4[1], g[0] <= max(1e-5, 2 * r4[0]))
        print(f"  {'':16} rms " + " ".join(f"{v:11.3e}        " for v in rms.values()) +
              f" criterion vs radix-4 (rms <= 1.1x, count <= 2x, max <= max(1e-5, 2x)): {ok}")


if __name__ == "__main__":
    main()
