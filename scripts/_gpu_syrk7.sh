#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/syrk7
timeout -k 10 300 python -u -m pytest tests/test_linalg_gpu.py -x -q --timeout 120 --timeout-method thread -k "syrk or cov" > gpurun_out/syrk7/pytest.log 2>&1 || { tail -30 gpurun_out/syrk7/pytest.log; exit 1; }
tail -1 gpurun_out/syrk7/pytest.log
python - <<'PY'
import torch, sys
sys.path.insert(0, ".")
from harp_amd.ops import linalg as LA
X = torch.rand(30016, 1000, device="cuda") * 2 - 1
fm = LA.FeatureMajor.from_rows(X)
G0 = LA.symmetrize_upper(LA.syrk_t(fm, variant=0))
G1 = LA.symmetrize_upper(LA.syrk_t(fm, variant=1))
print("spread==default", float((G0 - G1).abs().max()))
PY
for v in 0 1; do
  timeout -k 10 300 python scripts/bench_pca.py --variant $v --steps 2 > gpurun_out/syrk7/v$v.log 2>&1 || { tail -20 gpurun_out/syrk7/v$v.log; exit 1; }
  echo "v$v $(grep -o '"syrk_s_local": [0-9.e-]*' gpurun_out/syrk7/v$v.log)"
done
