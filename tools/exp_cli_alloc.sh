#!/bin/bash
# The drop-in CLI's first-call workspace growth and init stamps (RT_DEBUG 0x02 | 0x01), 5 runs.
cd "$GRAFT_REPO_ROOT" || exit 1
D=$(mktemp -d); python3 -c "import sys; sys.path.insert(0,'.'); import __graft_entry__ as g; p=g.import_pkg(); print(p.scenes.write_config('hm_verbatim', '$D'))" > /dev/null
for i in 1 2 3 4 5; do (cd $D && RT_DEBUG=3 timeout -k 5 60 "$GRAFT_REPO_ROOT/raytracer-ceng477-graphics-hw-1_amd/raytracer" hm_verbatim.xml --aa 1 --timing 2>&1 >/dev/null | grep -v '^$'); done
