# Build an A/B variant of the library: recompile the named sources with extra flags and link
# them with the current objects -> tts-sambert_hifigan_amd/libhifigan_hip.so.NAME (the C-ABI
# object, and with it the embedded source hash, is the tree's).  Run after build().
# usage: bash profiles/r03/variant.sh NAME "src1.hip src2.hip" -DFLAG=1 ...
set -e
NAME=$1; SRCS=$2; shift 2
P=tts-sambert_hifigan_amd; B=$P/build; V=/tmp/variant_$NAME; mkdir -p $V
OBJS=""
for o in conv_kernels conv_bf16x3 resblock_bf16x3 mrf_thin mrf_thin_mfma ups_bf16x3 probe hifigan_capi mel_kernels mel_capi; do
  if [[ " $SRCS " == *" $o.hip "* || " $SRCS " == *" $o.cpp "* ]]; then
    src=$P/csrc/$o.hip; [ -f $src ] || src=$P/csrc/$o.cpp
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -mcode-object-version=5 -O3 -std=c++17 -fPIC -Wall \
      -Wno-unused-result "$@" -c $src -o $V/$o.o
    OBJS="$OBJS $V/$o.o"
  else
    OBJS="$OBJS $B/$o.o"
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $OBJS -o $P/libhifigan_hip.so.$NAME
echo "built $P/libhifigan_hip.so.$NAME"
