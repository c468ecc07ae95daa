//go:build !mi355x

// The default (pure-Go) registration of the image-config secret analyzer:
// the init() of imgconf/secret/secret.go:17-19 moved behind the build tag, so
// that a `-tags mi355x` build registers secret_mi355x.go's constructor
// instead -- never both.  The one edit to secret.go is deleting its init().
package secret

import "github.com/aquasecurity/trivy/pkg/fanal/analyzer"

func init() {
	analyzer.RegisterConfigAnalyzer(analyzer.TypeImageConfigSecret, newSecretAnalyzer)
}
