"""`python -m grayscott_amd <settings.toml>`  (launch with torchrun for several ranks)."""
import sys

from .driver import julia_main

if __name__ == "__main__":
    sys.exit(julia_main(sys.argv[1:]))
