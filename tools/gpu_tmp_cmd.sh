for cfg in "1024 262144" "2048 131072" "512 262144"; do
  n=${cfg% *}; f=${cfg#* }
  echo "== N=$n"; timeout -k 10 200 python tools/ab_libs.py --rounds 7 --compare --n $n --frames $f head=abl/lib_head.so blim=abl/lib_blim.so || exit 1
done
