# round 4, session n: C4 / C5 of the committed build against the previous evidence build
# (final B showed C4 3 % below r4h on another box)
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_session.sh r4n ab:C4:ab_libs/evid.so,default:3 ab:C5:ab_libs/evid.so,default:2 || exit 1
