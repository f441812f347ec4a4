#!/bin/sh
# Builds the Node-API addon sail_napi.node against the image's Node headers (no node-gyp, no network).
set -e
cd "$(dirname "$0")"
mkdir -p build
NODE_INC=${NODE_INC:-/usr/include/node}
${CXX:-g++} -O2 -std=c++17 -shared -fPIC -DNODE_GYP_MODULE_NAME=sail_napi -DNAPI_VERSION=8 -I"$NODE_INC" \
  sail_napi.cc -o build/sail_napi.node -L../../lib -lsail_hip -Wl,-rpath,'$ORIGIN/../../../lib'
