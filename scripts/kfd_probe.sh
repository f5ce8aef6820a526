set -u
count() { for p in $(ls /proc | grep -E '^[0-9]+$'); do ls -l /proc/$p/fd 2>/dev/null | grep -qE '/dev/kfd|/dev/dri' && echo "$p $(tr '\0' ' ' < /proc/$p/cmdline | cut -c1-80)"; done; }
python -c "import torch, time; time.sleep(8)" & sleep 5; echo "== import torch"; count; wait
python -c "import torch, torch.distributed as d, time; time.sleep(8)" & sleep 5; echo "== import torch.distributed"; count; wait
python -c "import sys; sys.path.insert(0,'.'); from rnb_amd.config import gpu_memory_free_bytes as f; print(f()); import time; time.sleep(8)" & sleep 6; echo "== amdsmi free bytes"; count; wait
