"""Diagnostic: locate mismatches between the GPU batch and the C oracle at 1M x 1200."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch, hysteria_amd
from oracle.salamander_ref import COracle
co = COracle()
dev = torch.device("cuda:0")
L = 1200
for n in [int(a) for a in sys.argv[1:]] or [1 << 20]:
    inp = torch.empty(n * L, dtype=torch.uint8, device=dev)
    hysteria_amd.synth_stream(inp, n * L, 1, 0)
    salts = torch.empty(n, dtype=torch.int64, device=dev)
    hysteria_amd.synth_u64(salts, n, 2, 0)
    torch.cuda.synchronize()
    h_in = inp.cpu().numpy()
    ref_in = co.fill_stream(1, 0, n * L)
    bad_in = np.nonzero(h_in != ref_in)[0]
    print(n, "input mismatches:", bad_in.size, bad_in[:5])
    h_s = salts.cpu().numpy().view(np.uint64)
    print(n, "salt mismatches:", int((h_s != co.salts(2, 0, n)).sum()))
    o = hysteria_amd.SalamanderObfuscator(b"average_password", 0)
    for stride in (L + 8, 0):
        out = torch.empty(n * (L + 8), dtype=torch.uint8, device=dev)
        o.obfuscate_batch(inp, n, in_stride=L, len_uniform=L, salts=salts, out=out, out_stride=stride)
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        exp, _, _, _ = co.batch(True, b"average_password", n, ref_in, in_stride=L, len_uniform=L,
                                salts=co.salts(2, 0, n), out_cap=n * (L + 8))
        bad = np.nonzero(got != exp)[0]
        print(n, "stride", stride, "out mismatches:", bad.size)
        if bad.size:
            pk = np.unique(bad // (L + 8))
            print("  packets:", pk.size, pk[:20], "tiles:", np.unique(pk // 256)[:20])
            print("  first bytes:", bad[:10], "pos in pkt:", (bad % (L + 8))[:10])
            b0 = bad[0]
            print("  got", got[b0:b0+16], "exp", exp[b0:b0+16])
    o.close()
