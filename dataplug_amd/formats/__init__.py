"""Format plugins on the indexing path: FASTA, FASTQGZip (genomics), CSV (generic), VCF, GZipText."""
