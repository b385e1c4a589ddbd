"""grayscott_amd.parallel"""
