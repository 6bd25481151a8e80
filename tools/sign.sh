#!/bin/bash
# Detached GPG signatures of the native sources, like the reference's signed
# submissions (reference README.md:17-21: `gpg -ab main.cu`, *.asc force-added).
#
#   tools/sign.sh [--key KEYID] [--verify] [files...]
#
# Default file set: the lab programs and kernels (native/apps, native/src).
# Signatures are written next to each file as FILE.asc; *.asc is git-ignored,
# add them with `git add -f` when a signed submission is wanted.
set -euo pipefail
cd "$(dirname "$0")/.."
KEY=()
VERIFY=0
FILES=()
while [ $# -gt 0 ]; do
  case "$1" in
    --key) KEY=(--local-user "$2"); shift 2 ;;
    --verify) VERIFY=1; shift ;;
    *) FILES+=("$1"); shift ;;
  esac
done
if [ ${#FILES[@]} -eq 0 ]; then
  mapfile -t FILES < <(find native/apps native/src -type f \( -name '*.c' -o -name '*.cpp' -o -name '*.hip' -o -name '*.hpp' -o -name '*.h' \) | sort)
fi
command -v gpg >/dev/null || { echo "gpg not found" >&2; exit 2; }
for f in "${FILES[@]}"; do
  if [ $VERIFY -eq 1 ]; then
    gpg --verify "$f.asc" "$f"
  else
    gpg --batch --yes "${KEY[@]}" -ab "$f"
    echo "signed $f -> $f.asc"
  fi
done
