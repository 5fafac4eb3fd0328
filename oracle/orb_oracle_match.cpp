// matcher restatement (filled in later)
