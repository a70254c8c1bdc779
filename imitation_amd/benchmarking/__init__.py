"""Benchmark tooling (reference: benchmarking/): command generation, run collection,
normalised-score summaries with IQM and stratified-bootstrap CIs, probability of improvement."""
