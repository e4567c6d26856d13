set -o pipefail
bash tools/_r03e.sh && bash tools/_r03d.sh
