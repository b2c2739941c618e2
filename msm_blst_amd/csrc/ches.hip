// ches.hip -- CHES bucket-set pipeline (filled in below)
