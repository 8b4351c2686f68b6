"""Run ONE GEMM shape/layout through the tam.gemm routing, ``iters`` times
(for rocprofv3 --pmc passes; tools/gpu_r3_pmc.sh)."""
import sys

import torch

sys.path.insert(0, __file__.rsplit("/tools/", 1)[0])
from tiresias_amd.ops import _lib  # noqa: E402


def main():
    M, N, K = (int(x) for x in sys.argv[1:4])
    lay = sys.argv[4]
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    tile = int(sys.argv[6]) if len(sys.argv) > 6 else 256
    ak, bk = lay[0] == "K", lay[1] == "K"
    T = _lib.ops()
    dev = torch.device("cuda", 0)
    A = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    B = (torch.rand(K, N, device=dev) * 2 - 1).to(torch.bfloat16)
    a_ = A if ak else A.t().contiguous()
    b_ = B.t().contiguous() if bk else B
    c = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    T.gemm8p_policy(2, tile)         # force the 256^2 (or 128^2) p8 kernel, no split
    for _ in range(iters):
        T.gemm(a_, ak, b_, bk, c, 0, None, False, None, 1.0, False)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
