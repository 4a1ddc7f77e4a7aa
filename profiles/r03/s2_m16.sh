O=gpurun_out/s2m16; mkdir -p $O
bash profiles/r03/ab_env.sh s2m16/ab "HFG_MFMA16=1" "HFG_MFMA16=0" --streams 1 || exit 1
echo done
