#!/bin/bash
# Which in-process orderings of amdsmi (init/shutdown) and HIP (torch / sentinel) work?
cd "${GRAFT_REPO_ROOT:-.}"
run() {
  echo "--- $1"
  timeout -k 5 40 python -c "
import sys, time; sys.path.insert(0, '.')
import torch
from kubernetes_gpu_exporter_amd._native import load
n = load()
$2
print('BODY-DONE', flush=True)
" 2>&1 | tail -4
  echo "rc=${PIPESTATUS[0]}"
}
run "A: amdsmi init+shutdown, then torch" "n.read_backend('amdsmi'); x = torch.ones(4, device='cuda'); torch.cuda.synchronize(); print('torch ok', x.sum().item())"
run "B: torch first, then amdsmi init+shutdown, then torch" "x = torch.ones(4, device='cuda'); n.read_backend('amdsmi'); y = torch.ones(4, device='cuda') * 2; torch.cuda.synchronize(); print('torch ok', y.sum().item())"
run "C: python amdsmi init+shutdown, then torch" "import amdsmi; amdsmi.amdsmi_init(); amdsmi.amdsmi_shut_down(); x = torch.ones(4, device='cuda'); torch.cuda.synchronize(); print('torch ok')"
run "D: amdsmi engine with sentinel, stop, then torch" "
c = n.EngineConfig(); c.backend='amdsmi'; c.interval_s=0; c.serve_http=False; c.enable_sentinel=True; c.device_filter=[0]
e = n.Engine(c); e.start(); e.tick(); time.sleep(0.05); e.tick(); e.stop()
x = torch.ones(4, device='cuda'); torch.cuda.synchronize(); print('torch ok')"
run "E: torch init, engine with sentinel (amdsmi stays up), torch again" "
x = torch.ones(4, device='cuda')
c = n.EngineConfig(); c.backend='amdsmi'; c.interval_s=0; c.serve_http=False; c.enable_sentinel=True; c.device_filter=[0]
e = n.Engine(c); e.start(); e.tick(); time.sleep(0.05); e.tick()
y = torch.ones(4, device='cuda') * 3; torch.cuda.synchronize(); print('torch ok', y.sum().item()); e.stop()"
run "F: no torch GPU use, amdsmi only (exit hang?)" "n.read_backend('amdsmi')"
run "G: sysfs backend + sentinel only" "
c = n.EngineConfig(); c.backend='sysfs'; c.interval_s=0; c.serve_http=False; c.enable_sentinel=True; c.device_filter=[0]
e = n.Engine(c); e.start(); e.tick(); time.sleep(0.05); e.tick(); print(e.source_status()); e.stop()
x = torch.ones(4, device='cuda'); torch.cuda.synchronize(); print('torch ok')"
