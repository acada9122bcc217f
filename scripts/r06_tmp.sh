set -u
TAG=${TAG} TESTS="${TESTS:-}" LINES="${LINES:-}" LIBLINES="${LIBLINES:-}" bash scripts/ab_lines.sh || exit $?
