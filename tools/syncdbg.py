import os, sys, warnings, traceback
REPO = "/root/repo" if os.path.exists("/root/repo/bench.py") else os.getcwd()
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "self-supervise-sfm_amd"))
import torch, bench
dev = torch.device("cuda", 0)
model, _ = bench.build_model(dev)
n = 2
x = torch.rand(n, 3, 518, 518)
images = torch.cat([x, x])[None].to(dev)
def step():
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        return model(images, no_reloc_list=list(range(n)), reloc_list=list(range(n, 2 * n)), fix_rank=300)
step(); torch.cuda.synchronize()
def show(message, category, filename, lineno, file=None, line=None):
    print("SYNC:", message, flush=True)
    for fr in traceback.extract_stack()[:-1]:
        if "sailrecon_amd" in fr.filename or "bench" in fr.filename:
            print("    ", fr.filename.split("/")[-1], fr.lineno, fr.line, flush=True)
warnings.showwarning = show
torch.cuda.set_sync_debug_mode("warn")
step()
torch.cuda.set_sync_debug_mode(0)
print("done")
