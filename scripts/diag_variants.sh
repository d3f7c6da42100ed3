for v in librlamd.so librlamd_O1.so librlamd_u32.so; do
  echo "== $v"; RLAMD_LIB=rl-rust_amd/lib/$v timeout -k 10 200 python scripts/diag_private2.py 2>&1 | grep -E "case|first" | head -4 | cut -c1-200
done
