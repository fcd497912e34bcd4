__version__ = "1.0.0"   # the metadata version tag written to S3 (reference: dataplug/version.py)
