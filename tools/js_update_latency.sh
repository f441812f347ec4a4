#!/bin/bash
# Renderer.update() latency through the JS host with a cold and then a warm user code-object cache
# (tests/js/update_swap.js; profiles/r05_js_update_latency.jsonl). Needs an MI355X.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/jsupd; rm -rf $O; mkdir -p $O
export XDG_CACHE_HOME=$(pwd)/$O/xdg AMD_COMGR_CACHE=0
for label in cold warm; do
  timeout -k 10 300 node tests/js/update_swap.js $O/$label 40 24 4 5 || exit 3
  python3 -c "import json,sys; r=json.load(open(sys.argv[1])); r.pop('scene'); r['cache']=sys.argv[2]; print(json.dumps(r))" $O/$label.json $label >> $O/update_latency.jsonl || exit 4
done
cat $O/update_latency.jsonl
