# Same-box A/B of library variants on one legs.py leg, alternated 3 times, each variant with
# and without extra environment settings.
# usage (GPU box): bash profiles/r03/ab_legs.sh LEG "ENV1;ENV2" variant1 variant2 ...
# (ENV entries like "HFG_THIN_MFMA=1"; "-" = no extra setting)
LEG=$1; ENVS=$2; shift 2
L=tts-sambert_hifigan_amd/libhifigan_hip.so
cp $L /tmp/abl_keep.so
IFS=';' read -ra EV <<< "$ENVS"
for i in 1 2 3; do
  for v in "$@"; do
    for e in "${EV[@]}"; do
      cp $L.$v $L
      if [ "$e" = "-" ]; then r=$(timeout -k 10 120 python profiles/r03/legs.py $LEG 2>/dev/null | tail -1)
      else r=$(env $e timeout -k 10 120 python profiles/r03/legs.py $LEG 2>/dev/null | tail -1); fi
      [ -n "$r" ] || { cp /tmp/abl_keep.so $L; echo "FAILED $v $e"; exit 1; }
      echo "$i $v $e $r"
    done
  done
done
cp /tmp/abl_keep.so $L
