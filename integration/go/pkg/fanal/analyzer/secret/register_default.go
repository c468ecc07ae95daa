//go:build !mi355x

// The default (pure-Go) registration of the secret analyzer.  It is the
// init() of secret.go:44-47 moved behind the build tag, so that a
// `-tags mi355x` build registers the GPU post-analyzer (secret_mi355x.go)
// instead of this per-file analyzer -- never both.  The one edit to
// secret.go a maintainer makes is deleting its init().
package secret

import (
	"github.com/aquasecurity/trivy/pkg/fanal/analyzer"
	"github.com/aquasecurity/trivy/pkg/fanal/secret"
)

func init() {
	// The scanner will be initialized later via InitScanner()
	analyzer.RegisterAnalyzer(NewSecretAnalyzer(secret.Scanner{}, ""))
}
