for ab in 0 3 1 2 16 4 64; do echo "== ablate $ab"; timeout -k 10 120 python3 -u tools/h64_stamps.py $ab 2>&1 | grep "stage 0\|stage 2" | cut -c1-150 || exit 1; done
