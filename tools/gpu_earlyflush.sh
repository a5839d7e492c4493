set -o pipefail
for ef in 8 16 32 64 128 1000; do
  echo "ef=$ef"; TEMPI_EARLY_FLUSH=$ef timeout -k 10 120 tempi_amd/lib/halo_exchange 10 512 | cut -c 1-60,300-520 || exit 3
done
