"""TEST INFRASTRUCTURE (a checker, not product): the GPU demod's FFT (k_demod.hip
fft2048_wg: radix-8 / W2048 twiddles, radix-8 / W256, radix-8 / W32 and the quad's DPP
radix-4, fma twiddle products, and the fma the compiler contracts inside the radix-8
butterfly) restated in numpy float32, operation for operation.
tests/test_gpu_parity.py::test_demod_fft_equals_restated_transform pins it bit for bit to
the fused demod's spectra; tools/soft_floor.py compares its rounding with other fp32
transforms on the CPU."""
import numpy as np
f32 = np.float32
W = np.exp(-2j*np.pi*np.arange(2048)/2048)
Wr = W.real.astype(f32); Wi = W.imag.astype(f32)
C = f32(0.70710678118654752440)
def fmaf(a,b,c):
    """float32 fma, exactly: the product is exact in double; the double sum s = RN(p + c)
    rounds to the float RN(p + c) unless s is itself a float midpoint (double rounding),
    where the sign of the sum's error e (TwoSum) decides"""
    p = np.asarray(a, np.float64) * np.asarray(b, np.float64)
    c = np.asarray(c, np.float64)
    s = p + c
    bp = s - c
    e = (p - bp) + (c - (s - bp))
    mid = (s.view(np.uint64) & np.uint64(0x1FFFFFFF)) == np.uint64(0x10000000)
    s = np.where(mid & (e != 0), np.nextafter(s, np.where(e > 0, np.inf, -np.inf)), s)
    return s.astype(f32)
def cmul(ar, ai, wr, wi):
    return fmaf(ar, wr, -(ai*wi)), fmaf(ar, wi, ai*wr)
def dft8(ar, ai):  # ar, ai: lists of 8 arrays
    br=[None]*8; bi=[None]*8
    for j in range(4):
        br[j]=ar[j]+ar[j+4]; bi[j]=ai[j]+ai[j+4]
        br[j+4]=ar[j]-ar[j+4]; bi[j+4]=ai[j]-ai[j+4]
    # the W8^1 / W8^3 products: b5 = C s5, b7 = (C s7r, -C s7i)
    s5r, s5i = br[5]+bi[5], bi[5]-br[5]
    s7r, s7i = bi[7]-br[7], br[7]+bi[7]
    p7r, p7i = C*s7r, -(C*s7i)
    br[6], bi[6] = bi[6], -br[6]
    dr=[None]*8; di=[None]*8
    h=0
    dr[h]=br[h]+br[h+2]; di[h]=bi[h]+bi[h+2]
    dr[h+1]=br[h+1]+br[h+3]; di[h+1]=bi[h+1]+bi[h+3]
    dr[h+2]=br[h]-br[h+2]; di[h+2]=bi[h]-bi[h+2]
    tr=br[h+1]-br[h+3]; ti=bi[h+1]-bi[h+3]
    dr[h+3]=ti; di[h+3]=-tr
    # h = 4: b5 +- b7 -- the compiler contracts (k_demod.hip builds with fp-contract=fast):
    # the b5 product is fused, fma(C, s5, +-b7), the b7 product rounded first (found on the
    # GPU's own spectra, test_demod_fft_equals_restated_transform)
    Cv = lambda a: np.full_like(a, C)
    dr[4]=br[4]+br[6]; di[4]=bi[4]+bi[6]
    dr[5]=fmaf(Cv(s5r), s5r, p7r); di[5]=fmaf(Cv(s5i), s5i, p7i)
    dr[6]=br[4]-br[6]; di[6]=bi[4]-bi[6]
    tr=fmaf(Cv(s5r), s5r, -p7r); ti=fmaf(Cv(s5i), s5i, -p7i)
    dr[7]=ti; di[7]=-tr
    o_r=[None]*8; o_i=[None]*8
    pairs=[(0,4,0,1),(2,6,2,3),(1,5,4,5),(3,7,6,7)]
    for a,b,x,y in pairs:
        o_r[a]=dr[x]+dr[y]; o_i[a]=di[x]+di[y]
        o_r[b]=dr[x]-dr[y]; o_i[b]=di[x]-di[y]
    return o_r, o_i
def gpu_fft(x):
    """x: complex64 [..., 2048] -> complex64 X as fft2048_wg computes it"""
    xr = x.real.astype(f32); xi = x.imag.astype(f32)
    sh = x.shape[:-1]
    t = np.arange(256)
    # pass 1
    ar=[xr[..., t+256*m] for m in range(8)]; ai=[xi[..., t+256*m] for m in range(8)]
    ar, ai = dft8(ar, ai)
    for k in range(1,8):
        ar[k], ai[k] = cmul(ar[k], ai[k], Wr[(t*k)&2047], Wi[(t*k)&2047])
    exr = np.empty(sh+(2048,), f32); exi = np.empty(sh+(2048,), f32)
    for k in range(8):
        exr[..., k*256+t]=ar[k]; exi[..., k*256+t]=ai[k]
    # pass 2
    k1 = t>>5; tp = t&31
    ar=[exr[..., k1*256+tp+32*m] for m in range(8)]; ai=[exi[..., k1*256+tp+32*m] for m in range(8)]
    ar, ai = dft8(ar, ai)
    for k in range(1,8):
        ar[k], ai[k] = cmul(ar[k], ai[k], Wr[(8*(tp*k))&2047], Wi[(8*(tp*k))&2047])
    ex2r = np.empty(sh+(2048,), f32); ex2i = np.empty(sh+(2048,), f32)
    for k in range(8):
        ex2r[..., (k1*8+k)*32+tp]=ar[k]; ex2i[..., (k1*8+k)*32+tp]=ai[k]
    # pass 3
    g = t>>2; tq = t&3
    ar=[ex2r[..., g*32+tq+4*m] for m in range(8)]; ai=[ex2i[..., g*32+tq+4*m] for m in range(8)]
    ar, ai = dft8(ar, ai)
    for k in range(1,8):
        wr = np.where(tq>0, Wr[(64*(tq*k))&2047], f32(1)); wi = np.where(tq>0, Wi[(64*(tq*k))&2047], f32(0))
        nr, ni = cmul(ar[k], ai[k], wr, wi)
        ar[k] = np.where(tq>0, nr, ar[k]); ai[k] = np.where(tq>0, ni, ai[k])
    # pass 4: radix-4 across quads (lanes t: partner t^2 then t^1)
    def bfly(v, M):
        idx = t ^ M
        p = v[..., idx]
        sign = np.where(t & M, f32(-1), f32(1))
        return fmaf(sign, v, p)
    out = np.empty(sh+(2048,), np.complex64)
    b0 = (g>>3) + 8*(g&7) + 512*(((tq&1)<<1)|(tq>>1))
    for k in range(8):
        vr = bfly(ar[k], 2); vi = bfly(ai[k], 2)
        rot = tq == 3
        vr, vi = np.where(rot, vi, vr), np.where(rot, -vr, vi)
        vr = bfly(vr, 1); vi = bfly(vi, 1)
        out[..., b0 + 64*k] = vr + 1j*vi
    return out
