set -e
L=scripts/ab_libs/libflrl_rlv1.so,fl-rl-compression-mpi_amd/lib/libflrl.so
for k in runs32 longruns zero u8 upto4 upto12 upto24 lo4; do
  timeout -k 10 120 python scripts/ab_libs.py --op rl_encode --libs $L --kind $k --reps 15
done
