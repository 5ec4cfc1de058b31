#!/bin/bash
# Freeze the current tree (sources + built .so) into .snap/ so a queued gpurun call runs a consistent
# copy while the working tree keeps changing; .snap/gpurun_out points at the real gpurun_out.
# usage: bash tools/snap.sh   then   gpurun -- 'cd .snap && bash tools/<script>.sh'
set -e
cd /root/repo
# refuse a library older than its sources (a snapshot taken while `make` was relinking it is the likely
# cause of round 3's one unexplained abort)
so=asr-model_amd/asrx/libasrx.so
if [ -n "$(find asr-model_amd/csrc include -newer $so -type f | head -1)" ]; then
  echo "snap: $so is older than its sources; run make first" >&2; exit 1
fi
rm -rf .snap.new
mkdir .snap.new
tar --exclude=./.git --exclude=./gpurun_out --exclude=./.snap --exclude=./.snap.new --exclude=./asr-model_amd/build \
  --exclude=__pycache__ --exclude=.pytest_cache -cf - . | tar -xf - -C .snap.new
ln -sfn ../gpurun_out .snap.new/gpurun_out
rm -rf .snap
mv .snap.new .snap
