import json, sys, time
sys.path.insert(0, ".")
import numpy as np, torch
from novalsm_amd import crc32c as C
from bench import sst4k_layout
C.load(); assert C.load().nova_device_init() == 0
C.engine_set_enabled(1)
offs_np, lens_np, total = sst4k_layout(1024, 33)
img = torch.empty(total + 64, dtype=torch.uint8, device="cuda")
C.fill_splitmix64(img, 5)
offs = torch.from_numpy(offs_np.view(np.int64)).cuda(); lens = torch.from_numpy(lens_np.view(np.int32)).cuda()
C.write_trailers(img, offs, lens); torch.cuda.synchronize()
ok = torch.empty(1024, dtype=torch.uint8, device="cuda")
import ctypes
def cnt(tag):
    v = (ctypes.c_uint64 * 9)()
    C.load().nova_sst_engine_debug(v)
    print(tag, json.dumps(C.engine_counters()), "DBG why exited yv ygen0 quiet idle hostygen hyield consumed", list(v), flush=True)
for idle in (1000, 500000):
    C.engine_stop(); C.engine_set_idle_us(idle)
    cnt(f"idle={idle} after stop")
    C.queue_verify_blocks(img, offs, lens, ok)
    cnt("after queue call")
    time.sleep(0.005)
    cnt("5 ms later")
    s = torch.cuda.Stream(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    C.verify_blocks(img, offs, lens, stream=s, ok=ok); s.synchronize()
    print("plain call ms", (time.perf_counter() - t0) * 1e3)
    cnt("after plain")
    C.queue_verify_blocks(img, offs, lens, ok)
    cnt("after 2nd queue call")
