set -o pipefail
timeout -k 10 300 python tools/ab_libs.py --rounds 7 base=abl/lib_base.so winreg=abl/lib_winreg.so pf1=abl/lib_pf1.so pf0=abl/lib_pf0.so || exit 1
echo "== C3 features (SUB kernel)"; timeout -k 10 200 python tools/ab_libs.py --rounds 5 --features spectralCentroid,spectralFlatness,spectralSlope,spectralRolloff,spectralSpread,spectralSkewness,spectralKurtosis,loudness,perceptualSpread,perceptualSharpness base=abl/lib_base.so winreg=abl/lib_winreg.so pf1=abl/lib_pf1.so pf0=abl/lib_pf0.so || exit 1
