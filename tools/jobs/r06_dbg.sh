#!/bin/bash
cd /root/repo
for v in g8noslp; do echo "== variant $v"; timeout -k 10 200 python -u tools/ab_run.py abx/libuva_$v.so tools/dbg_dgelu.py 2>&1 | grep -v amdgpu.ids | grep dgelu; done
