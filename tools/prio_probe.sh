# developer probe: extraction / matching overlap under stream-placement knobs
# usage: bash tools/prio_probe.sh "ENV=.. ENV2=.." "ENV=.." ...
set -e -o pipefail
for cfg in "$@"; do
    echo "== $cfg"
    env $cfg timeout -k 10 200 python tools/overlap_probe.py 2>&1 | grep -v amdgpu.ids
done
