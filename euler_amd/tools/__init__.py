"""Command-line tools: JSON->Euler converter, shard service launcher, knn, console."""
