# round 4, session l: keep every C->V in registers on 802.11n (spill-free since r4k), 8 of 8 on
# 5G BG2
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_session.sh r4l ab:C3:ab_libs/keepall.so,default:3 ab:C4:ab_libs/keep8.so,default:2 || exit 1
