set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in librp_diag.so librp_diag_NOSTAMP.so librp_diag_NOTD.so librp_diag_BOTH.so librp_diag_LICM.so; do
  echo "== $v" >> gpurun_out/bisect.txt
  timeout -k 10 120 python -c "
import os,sys
sys.path[:0]=['.','raytracing-potato_amd']
os.environ['RP_LIB']='raytracing-potato_amd/lib/$v'
from rtpotato import scenes
from rtpotato.render import DeviceScene
from dataclasses import replace
sc,p=scenes.config_scene('C1')
ds=DeviceScene(sc)
try:
  _,_,st=ds.render(p); print('ok', st)
except Exception as e: print('ERR', e)
" >> gpurun_out/bisect.txt 2>&1 || exit 1
done
