#!/usr/bin/env python3
"""Drop-in for the reference's predict.py (same flags): see leastereo_amd/predict.py."""
import sys

from leastereo_amd.predict import main

if __name__ == "__main__":
    sys.exit(main())
