"""Host-input msm_compute wall time by size and by the host arrays' page alignment (diagnosis of the
slower ragged sizes)."""
import sys, os, time, statistics, json
sys.path[:0] = ["/root/repo", "/root/repo/webgpu-msm_amd"]
import numpy as np
import msm_amd as M
N = 1 << 20
pts = M.gen_points(N + 4096)
sc = M.gen_scalars(N + 4096, seed=5)
def t(p, s, runs=5, w=None):
    M.compute_msm_wire(p, s, window_size=w)
    ts = []
    for _ in range(runs):
        t0 = time.perf_counter(); M.compute_msm_wire(p, s, window_size=w); ts.append((time.perf_counter() - t0) * 1e3)
    return round(statistics.median(ts), 3)
def aligned(a):
    buf = np.empty(a.size + 1024, np.uint32)
    off = (-buf.ctypes.data % 4096) // 4
    out = buf[off:off + a.size].reshape(a.shape); out[:] = a; return out
WIN = os.environ.get("PROBE_WINDOWS") == "1"
cases = {
  "2^20 aligned": (aligned(pts[:N]), aligned(sc[:N])),
  "2^20 view +524": (pts[524:524 + N], sc[524:524 + N]),
  "2^20-524 aligned": (aligned(pts[:N - 524]), aligned(sc[:N - 524])),
  "2^20-524 view +524": (pts[524:N], sc[524:N]),
  "2^20-1 aligned": (aligned(pts[:N - 1]), aligned(sc[:N - 1])),
  "2^20+1 aligned": (aligned(pts[:N + 1]), aligned(sc[:N + 1])),
  "7*2^17 aligned": (aligned(pts[:7 << 17]), aligned(sc[:7 << 17])),
}
for r in range(2):
    for k, (p, s) in cases.items():
        for w in ((None, 14, 15) if WIN else (None,)):
            if WIN and "view" in k:
                continue
            print(json.dumps({"case": k, "round": r, "n": p.shape[0], "window": w, "ptr_mod_4096": p.ctypes.data % 4096,
                              "median_ms": t(p, s, w=w)}), flush=True)
