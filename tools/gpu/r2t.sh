set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/r2t_pytest.log 2>&1 && echo PYTEST_OK && \
timeout -k 10 200 python -u - > gpurun_out/r2t_kabsch.log 2>&1 <<'PY' && echo KABSCH_OK
import os, sys, numpy as np, torch
sys.path[:0] = ["ssf-slam_amd", "."]
import ssf
g = np.load("tests/golden/kabsch_ref.npz")
fe = ssf.Frontend(64, device=0)
for c in range(4):
    src, dst = g[f"src{c}"], g[f"dst{c}"]
    for dt in (torch.float64, torch.float32):
        pts = torch.from_numpy(np.ascontiguousarray(dst)).to("cuda", dt)
        fl = torch.from_numpy(np.ascontiguousarray(src - dst)).to("cuda", dt)
        off, h_off = ssf.frame_offsets([len(dst)], torch.device("cuda", 0))
        ones = torch.ones(len(dst), dtype=torch.uint8, device="cuda")
        out, _ = fe.mask_pose(pts, fl, off, h_off, mode="given", mask_in=ones)
        o = out[0].cpu().numpy()
        print(c, dt, "dR", np.abs(o[7:16].reshape(3, 3) - g[f"R{c}"]).max(), "dt", np.abs(o[0:3] - g[f"t{c}"]).max())
PY
