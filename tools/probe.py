"""Quick throughput probe: scene, W, H, spp, bounces -> Msamples/s (kernel events)."""
import sys, os, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "montecarlo-pathtracing_amd"))
import numpy as np
import mcpt

sid = int(sys.argv[1]) if len(sys.argv) > 1 else 6
W = int(sys.argv[2]) if len(sys.argv) > 2 else 1920
H = int(sys.argv[3]) if len(sys.argv) > 3 else 1080
S = int(sys.argv[4]) if len(sys.argv) > 4 else 16
B = int(sys.argv[5]) if len(sys.argv) > 5 else 8
r = mcpt.Renderer(0)
sc = mcpt.Scene.reference(sid)
r.upload_scene(sc)
r.set_target(W, H)
ipv, iv = mcpt.camera_canonical(W, H)
r.render(ipv, iv, 1, 1, 0.0, B, 1.0, 0)
r.synchronize()
for it in range(3):
    t = time.time()
    r.render(ipv, iv, 1 + it * S, S, 0.0, B, 1.0, 0)
    ms = r.last_render_ms()
    dt = time.time() - t
    print(f"scene {sid} {W}x{H} S={S} B={B}: kernel {ms:.2f} ms  {W*H*S/ms/1e3:.1f} Msamples/s  (wall {dt*1e3:.1f} ms)", flush=True)
ev = r.render_counted(ipv, iv, 1, 2, 0.0, B, 1.0, 0)
print("events/sample", dict(zip(mcpt.EVENT_NAMES, (ev / (W * H * 2)).round(3))))
print("bytes/sample", float((ev * mcpt.Renderer.event_bytes()).sum() / (W * H * 2)))
