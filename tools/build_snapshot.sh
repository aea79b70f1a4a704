#!/bin/bash
# Build in a snapshot of the source tree, so sources can be edited while it compiles: copies the
# tree (no .git, results or libraries; built objects kept, mtimes preserved) to /tmp/bt_<name>, runs
# `make <args>` there and copies the libraries it built back into bling_amd/_lib.  For experiment
# builds; the committed tree is built in place (make all) so that `make -n all` has nothing to do.
#   [PRE=cmd] bash tools/build_snapshot.sh NAME make-args...      e.g. NAME=x variant V=x DEFS=-D...
set -e
NAME=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
BT=/tmp/bt_$NAME
rm -rf $BT/bling_amd/_lib
mkdir -p $BT
(cd $ROOT && tar --exclude=./.git --exclude=./gpurun_out --exclude=./bling_amd/_lib --exclude=./profiles \
     --exclude=./oracle/_build -cf - .) | (cd $BT && tar xf -)
# PRE: a command run in the snapshot before make (e.g. restore one file from HEAD)
[ -n "$PRE" ] && (cd $BT && eval "$PRE")
touch /tmp/bt_stamp_$NAME
cd $BT && make -j8 "$@"
for f in $BT/bling_amd/_lib/libbling_hip*.so; do
  [ "$f" -nt /tmp/bt_stamp_$NAME ] && cp -p "$f" $ROOT/bling_amd/_lib/
done
echo "snapshot build $NAME done"
