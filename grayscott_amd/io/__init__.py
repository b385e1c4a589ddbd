"""grayscott_amd.io"""
